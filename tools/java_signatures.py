"""Method signatures of Java classes, parsed from source (no JDK in the image): the check that
the JVM adapters (electionguard-remote_amd/jvm) implement the reference's interfaces with the exact
parameter types, order, @Nullable markers and return types the reference uses.

    python tools/java_signatures.py --make-fixture   # (re)writes tests/golden/reference_signatures.json
                                                     # from /root/reference (DecryptingTrusteeIF as
                                                     # RemoteDecryptingTrusteeProxy implements it, and
                                                     # the call sites in RunRemoteDecryptingTrustee)
The fixture holds data only: method names, return types, parameter types, annotations and the call
sites' argument counts / null positions (no reference source text)."""
from __future__ import annotations

import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
FIXTURE = ROOT / "tests" / "golden" / "reference_signatures.json"
REF = Path("/root/reference/src/main/java/electionguard/decrypt")


def _strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def _split_params(s: str):
    """Split a parameter list at top-level commas (generics nest)."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [p.strip() for p in out]


def _param(p: str):
    """'@Nullable ElementModQ nonce' -> {'type': 'ElementModQ', 'nullable': True}"""
    ann = re.findall(r"@(\w+)", p)
    p = re.sub(r"@\w+(\([^)]*\))?", " ", p)
    p = re.sub(r"\bfinal\b", " ", p).strip()
    typ = re.sub(r"\s+", "", p.rsplit(None, 1)[0])
    return {"type": typ, "nullable": "Nullable" in ann}


def override_methods(src: str):
    """name -> {'returns', 'params'} of every @Override public method."""
    src = _strip_comments(src)
    pat = re.compile(r"@Override\s+public\s+([\w<>\[\], ?]+?)\s+(\w+)\s*\(([^)]*)\)", re.S)
    out = {}
    for m in pat.finditer(src):
        ret, name, params = re.sub(r"\s+", "", m.group(1)), m.group(2), m.group(3)
        out[name] = {"returns": ret, "params": [_param(p) for p in _split_params(params)]}
    return out


def delegate_calls(src: str):
    """name -> list of (argument count, indices of literal-null arguments) of delegate.<name>(...) calls."""
    src = _strip_comments(src)
    out = {}
    for m in re.finditer(r"delegate\.(\w+)\s*\(", src):
        i, depth, args, cur = m.end(), 1, [], ""
        while depth:
            ch = src[i]
            if ch in "([":
                depth += 1
            elif ch in ")]":
                depth -= 1
                if depth == 0:
                    break
            if ch == "," and depth == 1:
                args.append(cur)
                cur = ""
            else:
                cur += ch
            i += 1
        args.append(cur)
        args = [a.strip() for a in args if a.strip()]
        out.setdefault(m.group(1), []).append({"nargs": len(args),
                                               "null_args": [k for k, a in enumerate(args) if a == "null"]})
    return out


def compare(impl: dict, ref: dict, calls: dict):
    """-> list of human-readable mismatches between an implementation's methods and the reference's."""
    errs = []
    for name, want in ref.items():
        got = impl.get(name)
        if got is None:
            errs.append(f"{name}: missing")
            continue
        if got["returns"] != want["returns"]:
            errs.append(f"{name}: returns {got['returns']}, reference {want['returns']}")
        if [p["type"] for p in got["params"]] != [p["type"] for p in want["params"]]:
            errs.append(f"{name}: parameters {[p['type'] for p in got['params']]}, reference "
                        f"{[p['type'] for p in want['params']]}")
        if [p["nullable"] for p in got["params"]] != [p["nullable"] for p in want["params"]]:
            errs.append(f"{name}: @Nullable at {[i for i, p in enumerate(got['params']) if p['nullable']]}, "
                        f"reference {[i for i, p in enumerate(want['params']) if p['nullable']]}")
        for c in calls.get(name, []):  # the reference's own call sites must fit the implementation
            if c["nargs"] != len(got["params"]):
                errs.append(f"{name}: the reference calls it with {c['nargs']} arguments")
            for k in c["null_args"]:
                if k < len(got["params"]) and not got["params"][k]["nullable"]:
                    errs.append(f"{name}: the reference passes null as argument {k}, which is not @Nullable")
    return errs


def make_fixture() -> dict:
    proxy = (REF / "RemoteDecryptingTrusteeProxy.java").read_text()
    server = (REF / "RunRemoteDecryptingTrustee.java").read_text()
    return {
        "source": "DecryptingTrusteeIF as implemented by RemoteDecryptingTrusteeProxy.java:32-115; delegate calls "
                  "in RunRemoteDecryptingTrustee.java:189-193,227-232 (electionguard-remote, read-only reference)",
        "DecryptingTrusteeIF": override_methods(proxy),
        "delegate_calls": delegate_calls(server),
    }


if __name__ == "__main__":
    if "--make-fixture" in sys.argv:
        FIXTURE.write_text(json.dumps(make_fixture(), indent=1) + "\n")
        print("wrote", FIXTURE)
