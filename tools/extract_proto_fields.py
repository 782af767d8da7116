"""Extract the reference's wire format from its own ``.proto`` files into data.

    python tools/extract_proto_fields.py            # writes tests/golden/reference_proto_fields.json
    python tools/extract_proto_fields.py --check    # exit 1 if the committed JSON differs

Reads /root/reference/src/main/proto/*.proto (read-only; the reference's IDL, e.g.
decrypting_trustee_rpc.proto:9-45, common.proto:8-48, common_rpc.proto:6-12) and records, per
file: imports, package and every message's fields (name, number, scalar/message type, label,
type name), reserved numbers, and every service's methods with their request/response types.
``protoc`` is not in the image, so this is a small parser for the proto3 subset those files use
(messages without nesting, ``repeated``, ``reserved``, services of unary rpcs, ``//`` comments).

The output is DATA -- field tables, not source -- and tests/test_remote_wire.py compares
``electionguard.remote.POOL`` (the hand-built descriptors the trustee server and proxy speak) with
it in both directions.
"""
import argparse
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
REF_PROTO = Path("/root/reference/src/main/proto")
OUT = ROOT / "tests" / "golden" / "reference_proto_fields.json"

# proto3 scalar keywords -> google.protobuf FieldDescriptorProto.Type names
SCALARS = {
    "double": "TYPE_DOUBLE", "float": "TYPE_FLOAT", "int64": "TYPE_INT64", "uint64": "TYPE_UINT64",
    "int32": "TYPE_INT32", "fixed64": "TYPE_FIXED64", "fixed32": "TYPE_FIXED32", "bool": "TYPE_BOOL",
    "string": "TYPE_STRING", "bytes": "TYPE_BYTES", "uint32": "TYPE_UINT32", "sfixed32": "TYPE_SFIXED32",
    "sfixed64": "TYPE_SFIXED64", "sint32": "TYPE_SINT32", "sint64": "TYPE_SINT64",
}

_TOKEN = re.compile(r'"[^"]*"|[A-Za-z_][\w.]*|\d+|[{}();=,\[\]<>]')


def _tokens(text: str):
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return _TOKEN.findall(text)


def parse_proto(text: str) -> dict:
    """-> {"syntax", "package", "imports", "messages": {name: {"fields": [...], "reserved": [...]}},
    "services": {name: [{"name", "input", "output"}]}}; type names as written (resolved later)."""
    t = _tokens(text)
    out = {"syntax": None, "package": None, "imports": [], "messages": {}, "services": {}}
    i = 0

    def expect(tok):
        nonlocal i
        if t[i] != tok:
            raise ValueError(f"expected {tok!r} at token {i}, got {t[i]!r}")
        i += 1

    def skip_statement():
        nonlocal i
        while t[i] != ";":
            i += 1
        i += 1

    while i < len(t):
        w = t[i]
        if w == ";":
            i += 1
        elif w == "syntax":
            i += 2
            out["syntax"] = t[i].strip('"')
            i += 1
            expect(";")
        elif w == "package":
            out["package"] = t[i + 1]
            i += 2
            expect(";")
        elif w == "import":
            i += 1
            if t[i] in ("public", "weak"):
                i += 1
            out["imports"].append(t[i].strip('"'))
            i += 1
            expect(";")
        elif w == "option":
            skip_statement()
        elif w == "message":
            name = t[i + 1]
            i += 2
            expect("{")
            fields, reserved = [], []
            while t[i] != "}":
                if t[i] == ";":
                    i += 1
                elif t[i] == "reserved":
                    i += 1
                    while t[i] != ";":
                        if t[i].isdigit():
                            lo = int(t[i])
                            hi = lo
                            if t[i + 1] == "to":
                                hi = int(t[i + 2])
                                i += 2
                            reserved.append([lo, hi + 1])  # half-open, as DescriptorProto.ReservedRange
                        elif t[i].startswith('"'):
                            reserved.append(t[i].strip('"'))
                        i += 1
                    i += 1
                elif t[i] == "option":
                    skip_statement()
                elif t[i] in ("message", "enum", "oneof", "map"):
                    raise ValueError(f"{t[i]} inside message {name}: not used by the reference, not parsed")
                else:
                    label = "LABEL_OPTIONAL"
                    if t[i] in ("repeated", "optional"):
                        label = "LABEL_REPEATED" if t[i] == "repeated" else "LABEL_OPTIONAL"
                        i += 1
                    ftype, fname = t[i], t[i + 1]
                    i += 2
                    expect("=")
                    num = int(t[i])
                    i += 1
                    if t[i] == "[":
                        while t[i] != "]":
                            i += 1
                        i += 1
                    expect(";")
                    fields.append({"name": fname, "number": num, "label": label,
                                   "type": SCALARS.get(ftype, "TYPE_MESSAGE"),
                                   "type_name": None if ftype in SCALARS else ftype})
            i += 1
            out["messages"][name] = {"fields": fields, "reserved": reserved}
        elif w == "service":
            name = t[i + 1]
            i += 2
            expect("{")
            methods = []
            while t[i] != "}":
                if t[i] == "rpc":
                    m = t[i + 1]
                    i += 2
                    expect("(")
                    if t[i] == "stream":
                        raise ValueError("streaming rpcs are not used by the reference")
                    req = t[i]
                    i += 1
                    expect(")")
                    expect("returns")
                    expect("(")
                    resp = t[i]
                    i += 1
                    expect(")")
                    if t[i] == "{":
                        depth = 0
                        while True:
                            depth += {"{": 1, "}": -1}.get(t[i], 0)
                            i += 1
                            if depth == 0:
                                break
                    methods.append({"name": m, "input": req, "output": resp})
                else:
                    i += 1
            i += 1
            out["services"][name] = methods
        elif w == "enum":
            raise ValueError("top-level enums are not used by the reference's trustee protos")
        else:
            raise ValueError(f"unexpected token {w!r}")
    return out


def _resolve(files: dict) -> None:
    """Message type names -> fully qualified ('.Name' with no package, '.pkg.Name' with one),
    looked up in the file itself and its imports, as protoc resolves them."""
    def fq(name, fn):
        if name.startswith("."):
            return name
        if name.startswith("google.protobuf."):  # a well-known type from an imported google/protobuf/*.proto
            if any(imp.startswith("google/protobuf/") for imp in files[fn]["imports"]):
                return "." + name
        for cand in [fn] + files[fn]["imports"]:
            if cand in files and name in files[cand]["messages"]:
                pkg = files[cand]["package"]
                return f".{pkg}.{name}" if pkg else f".{name}"
        raise ValueError(f"{fn}: type {name} not found in the file or its imports")

    for fn, f in files.items():
        for m in f["messages"].values():
            for fl in m["fields"]:
                if fl["type_name"]:
                    fl["type_name"] = fq(fl["type_name"], fn)
        for methods in f["services"].values():
            for me in methods:
                me["input"], me["output"] = fq(me["input"], fn), fq(me["output"], fn)


def extract(proto_dir: Path = REF_PROTO) -> dict:
    files = {p.name: parse_proto(p.read_text()) for p in sorted(proto_dir.glob("*.proto"))}
    if not files:
        raise FileNotFoundError(f"no .proto files under {proto_dir}")
    _resolve(files)
    return {"source": "JohnLCaron/electionguard-remote src/main/proto (extracted by tools/extract_proto_fields.py)",
            "files": files}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--proto-dir", default=str(REF_PROTO))
    ap.add_argument("--out", default=str(OUT))
    ap.add_argument("--check", action="store_true", help="compare with the committed JSON instead of writing it")
    a = ap.parse_args(argv)
    data = extract(Path(a.proto_dir))
    text = json.dumps(data, indent=1, sort_keys=True) + "\n"
    if a.check:
        same = Path(a.out).read_text() == text
        print("reference_proto_fields.json matches the reference's .proto files" if same else
              "reference_proto_fields.json DIFFERS from the reference's .proto files")
        return 0 if same else 1
    Path(a.out).write_text(text)
    n = sum(len(f["messages"]) for f in data["files"].values())
    print(f"wrote {a.out}: {len(data['files'])} files, {n} messages")
    return 0


if __name__ == "__main__":
    sys.exit(main())
