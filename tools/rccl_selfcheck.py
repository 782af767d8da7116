"""RCCL self-check of the multi-GPU exchange on whatever GPUs one box has.

The exchange runs inside libeg_hip.so on its own HIP runtime (eg_comm_init /
eg_comm_all_valid / eg_tally_allgather_fold, electionguard.distributed.TallyExchange): a rank
verifies + tallies its ballots into a libeg device buffer, the verdict is an RCCL all-reduce(min)
and the partial tallies one ncclAllGather folded mod p on rank 0's GPU.  The process never brings
up a second GPU framework (torch is used only for its CPU gloo group: the RCCL id and a reference
gather of host copies).  Every rank's fold is checked against CPython products of the host copies.
RCCL refuses two ranks on one device, so on a 1-GPU box this runs at world size 1.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \\
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
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.core import productionGroup
    from electionguard.distributed import TallyExchange
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
    d_cts, d_rp, d_cp = (G.to_device(x) for x in (eb.cts, eb.rproof, eb.cproof))
    d_oks, d_okc = G.device_zeros((nb, man.nsel)), G.device_zeros((nb, man.n_contests))
    d_tal = G.device_zeros((man.n_real, 2, 512))
    Verifier(G, key, qbar, man).verify_device(d_cts.ptr, d_rp.ptr, d_cp.ptr, nb, d_oks.ptr, d_okc.ptr, d_tal.ptr)
    xch = TallyExchange(G, dist, world, rank, "rccl")
    ok = xch.all_valid(G.all_nonzero(d_oks) and G.all_nonzero(d_okc))
    folded = xch.fold(d_tal, man.n_real)
    # reference: host copies gathered over gloo, folded with CPython
    host_parts = [torch.empty((man.n_real, 2, 512), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(host_parts, torch.from_numpy(d_tal.download()))
    parts = np.stack([h.numpy() for h in host_parts])
    ok_fold = True
    if rank == 0:
        for s in range(man.n_real):
            for c in range(2):
                acc = 1
                for r in range(world):
                    acc = acc * int.from_bytes(parts[r, s, c].tobytes(), "big") % G.p
                ok_fold &= int.from_bytes(folded[s, c].tobytes(), "big") == acc
    xch.close()
    res = {"rank": rank, "world": world, "exchange": xch.collective, "verdict_all_valid": bool(ok),
           "fold_matches_cpython": ok_fold}
    print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok and ok_fold else 1


if __name__ == "__main__":
    sys.exit(main())
