"""A/B of the constant-time encryption tables' radix width (EG_CT_WINDOW, eg_ctx_set_ct_encrypt).

    python tools/ab_ct_window.py            # parent: one child process per width (read at ctx creation)
Each child encrypts the same 10k configs[1]-shape ballots, device-resident, in both modes and
prints the rates; the constant-time bytes must equal the default mode's.  A w-bit table costs
ceil(256/w) multiplies per fixed-base term, each with a masked scan of 2^w entries."""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))


def child(nb=10_000, reps=3):
    import torch
    torch.cuda.init()
    from electionguard.ballot import ElectionKey, Manifest, batch_encryption_device, random_scalars, random_votes
    from electionguard.core import productionGroup
    from electionguard.keyceremony import key_ceremony
    G = productionGroup(0)
    man = Manifest(4, 5, 1)
    _, K = key_ceremony(G, 3, 3, seed=5)
    key = ElectionKey(G, K, window_bits=22)
    rng = np.random.default_rng(5)
    dev = torch.device("cuda", 0)
    dv, dsn, dcn = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in
                    (random_votes(rng, man, nb), random_scalars(rng, (nb, man.nsel, 4), G.q),
                     random_scalars(rng, (nb, man.n_contests), G.q)))
    outs = {}
    res = {"ct_window": int(os.environ.get("EG_CT_WINDOW", "6"))}
    for ct in (False, True):
        G.ct_encrypt = ct
        o = [torch.empty(s, dtype=torch.uint8, device=dev) for s in
             ((nb, man.nsel, 2, 512), (nb, man.nsel, 4, 32), (nb, man.n_contests, 2, 32))]
        run = lambda: batch_encryption_device(G, key, 77, man, nb, dv.data_ptr(), dsn.data_ptr(), dcn.data_ptr(),
                                              *(x.data_ptr() for x in o))
        run()
        best = None
        for _ in range(reps):
            t = time.perf_counter()
            run()
            best = min(best or 1e9, time.perf_counter() - t)
        outs[ct] = o
        res["ct" if ct else "default"] = round(nb / best, 1)
    G.ct_encrypt = False
    res["same_bytes"] = all(bool(torch.equal(a, b)) for a, b in zip(outs[False], outs[True]))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
        sys.exit(0)
    rc = 0
    for w in (5, 6, 7):
        r = subprocess.run([sys.executable, __file__, "child"], env=dict(os.environ, EG_CT_WINDOW=str(w)), timeout=600)
        rc = rc or r.returncode
    sys.exit(rc)
