"""Report which proof conventions an upstream-produced record uses (see electionguard/formats.py):
verifies its wire-layout ballots and trustee shares on the GPU under every combination of the hash
pre-image hex form, the response sign and the pre-image order.

    python tools/pin_format.py record.json        # prints one JSON line per combination, then the verdict
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))


def main(argv):
    if len(argv) != 1:
        sys.exit(__doc__)
    from electionguard.core import productionGroup
    from electionguard.formats import pin_formats, summarize
    rec = json.loads(Path(argv[0]).read_text())
    res = pin_formats(productionGroup(0), rec)
    for r in res:
        print(json.dumps(r))
    s = summarize(res)
    print("pinned:" if s["response"] not in (None, "undetermined") and s["preimage"] not in (None, "undetermined")
          else "not pinned:", json.dumps(s))
    return 0 if s["response"] not in (None, "undetermined") and s["preimage"] not in (None, "undetermined") else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
