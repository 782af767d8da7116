"""Constant-time schedules (eg_ctx_set_ct_pow), measured: for every exponentiation layout, one batch per
exponent class -- all zero, all ones (2^256 - 1), random -- each its own kernel dispatch, with the
switch off and on.  Run under rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace (tools/gpu_r05.sh
ctpmc): the per-dispatch VALU instruction count of the constant-time dispatches must not depend on the
exponent class, while the variable-time ones do (sliding-window skips, zero-digit skips).  Also prints
the wall rate of each batch (the rate cost of the switch).  Dispatch order is printed on stdout so the
counter rows can be matched: tools/ct_schedule_summary.py does that.

    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -d OUT -o run -- python3 tools/ct_schedule.py"""
import json
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))

from electionguard.core import productionGroup  # noqa: E402


def main():
    G = productionGroup(0)
    q = G.q
    rng = random.Random(3)
    fb12 = G.fixed_base(pow(G.g, rng.randrange(q), G.p), 12)
    classes = {"zero": lambda: 0, "ones": lambda: 2**256 - 1, "random": lambda: rng.randrange(q)}
    layouts = [("per-wave powP right to left", 256), ("per-wave powP", 512), ("16-lane powP", 3000),
               ("8-lane powP", 9000), ("per-wave fixed-base 12-bit", 256)]
    log = []
    for ct in (False, True):
        G.ct_pow = ct
        for name, n in layouts:
            bases = [rng.randrange(G.p) for _ in range(n)]
            for cls, f in classes.items():
                exps = [f() for _ in range(n)]
                t = time.perf_counter()
                if "fixed" in name:
                    fb12.pow_batch(exps)
                else:
                    G.powP_batch(bases, exps)
                dt = time.perf_counter() - t
                rec = {"seq": len(log), "ct": ct, "layout": name, "n": n, "exponents": cls, "per_s": round(n / dt, 1)}
                log.append(rec)
                print(json.dumps(rec), flush=True)
    G.ct_pow = False


if __name__ == "__main__":
    main()
