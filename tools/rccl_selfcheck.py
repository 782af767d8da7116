"""RCCL self-check of the multi-GPU exchange on whatever GPUs one box has.

bench.py only initialises torch.distributed when WORLD_SIZE > 1, and RCCL refuses two
ranks on one device, so a 1-GPU box never runs the nccl (= RCCL) collectives of the
N > 1 bench.  This tool runs them at any world size, including 1, on the same objects the
bench uses: a libeg_hip.so verify + tally writes the partial tally into a torch device
tensor (two HIP runtimes in one process: torch's bundled one and the system one that
libeg_hip.so links), then all_reduce(MIN) of the verdict and all_gather_into_tensor of the
partial tallies go over RCCL, and rank 0 folds them mod p on its GPU.  Every rank checks
the fold against a fold of host copies gathered over a separate gloo group.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29541 tools/rccl_selfcheck.py
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))


def main():
    import torch
    import torch.distributed as dist

    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    gloo = dist.new_group(backend="gloo")
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.core import productionGroup
    from electionguard.keyceremony import key_ceremony

    G = productionGroup(local)
    man = Manifest(4, 5, 1)
    _, K = key_ceremony(G, 3, 3, seed=11)
    key = ElectionKey(G, K, window_bits=12)
    rng = np.random.default_rng(500 + rank)
    nb = 300
    votes = random_votes(rng, man, nb)
    qbar = 31337
    eb = batch_encryption(G, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), G.q),
                          random_scalars(rng, (nb, man.n_contests), G.q))
    dev = torch.device("cuda", local)
    d_cts, d_rp, d_cp = (torch.from_numpy(x).to(dev) for x in (eb.cts, eb.rproof, eb.cproof))
    d_oks = torch.zeros((nb, man.nsel), dtype=torch.uint8, device=dev)
    d_okc = torch.zeros((nb, man.n_contests), dtype=torch.uint8, device=dev)
    d_tal = torch.zeros((man.n_real, 2, 512), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    Verifier(G, key, qbar, man).verify_device(d_cts.data_ptr(), d_rp.data_ptr(), d_cp.data_ptr(), nb,
                                              d_oks.data_ptr(), d_okc.data_ptr(), d_tal.data_ptr())
    G.sync()
    # RCCL: verdict all_reduce(MIN) and the partial-tally all-gather on device tensors
    flag = torch.tensor([int(bool(d_oks.all().item() and d_okc.all().item()))], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    gathered = torch.empty((world * man.n_real, 2, 512), dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, d_tal.contiguous())
    torch.cuda.synchronize()
    parts = gathered.cpu().numpy().reshape(world, man.n_real, 2, 512)
    # reference exchange over gloo with host copies
    host_parts = [torch.empty((man.n_real, 2, 512), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(host_parts, d_tal.cpu(), group=gloo)
    want = np.stack([h.numpy() for h in host_parts])
    ok_gather = bool(np.array_equal(parts, want))
    # fold mod p on the GPU and compare with CPython products of the gathered partials
    g = np.ascontiguousarray(np.transpose(parts, (1, 2, 0, 3))).reshape(-1, 512)
    folded = G.prodP_groups(g, man.n_real * 2, world).reshape(man.n_real, 2, 512)
    ok_fold = True
    for s in range(man.n_real):
        for c in range(2):
            acc = 1
            for r in range(world):
                acc = acc * int.from_bytes(parts[r, s, c].tobytes(), "big") % G.p
            ok_fold &= int.from_bytes(folded[s, c].tobytes(), "big") == acc
    res = {"rank": rank, "world": world, "verdict_all_valid": bool(flag.item()), "rccl_all_gather_matches_gloo": ok_gather,
           "fold_matches_cpython": ok_fold}
    print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if all(v for k, v in res.items() if k not in ("rank", "world")) else 1


if __name__ == "__main__":
    sys.exit(main())
