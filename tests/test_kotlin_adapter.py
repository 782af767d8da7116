"""CPU: the L1 drop-in (GpuProductionGroupContext.kt) against the upstream GroupContext / ElementModP
members, without kotlinc.

The adapter implements the upstream interfaces by delegation and overrides only the hot-path
members (plus the constructors and constants that must hand out GPU elements).  The upstream
member list is restated in tests/golden/upstream_group_api.json (the jar is absent: UNPINNED).
Checked here: every override names a member of that list with its parameter and return types;
every hot-path member is overridden and reaches the deferred algebra (host/electionguard.hpp
Deferred, restated in Kotlin); every ElementModP argument is wrapped into a GPU element before it
reaches the algebra (an upstream element passed in must not escape it); every ElementModP result is
a GPU element; the element constructors and constants wrap.  Mutations must be caught."""
import json
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
KT = ROOT / "electionguard-remote_amd" / "jvm" / "src" / "main" / "kotlin" / "electionguard" / "gpu" / \
    "GpuProductionGroupContext.kt"
API = json.loads((ROOT / "tests" / "golden" / "upstream_group_api.json").read_text())


def _classes(src: str) -> dict:
    """class name -> (delegated interface, body text) for `class X(...) : Iface by y { body }`."""
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for m in re.finditer(r"\bclass\s+(\w+)\s*(?:internal\s+constructor\s*)?\(((?:(?!\bclass\b).)*?)\)\s*:\s*(\w+)"
                         r"\s+by\s+[\w.()]+\s*\{", src, flags=re.S):
        depth, i = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        out[m.group(1)] = (m.group(3), src[m.end():i - 1])
    return out


def _overrides(body: str) -> dict:
    """name -> {kind, params, names, returns|type, expr} of each `override val|fun` in a class body."""
    res = {}
    for m in re.finditer(r"override\s+((?:infix\s+|operator\s+)*)(val|fun)\s+([\w<>.]+?)\s*(\((.*?)\))?\s*:\s*"
                         r"([\w<>?]+)\s*(?:get\(\)\s*)?=\s*([^\n]+)", body):
        kind, name, params, typ, expr = m.group(2), m.group(3), m.group(5), m.group(6), m.group(7)
        ent = {"kind": kind, "expr": expr.strip()}
        if kind == "val":
            ent["type"] = typ
        else:
            ps = [p for p in params.split(",") if p.strip()] if params else []
            ent["params"] = [p.split(":")[1].strip() for p in ps]
            ent["names"] = [p.split(":")[0].strip() for p in ps]
            ent["returns"] = typ
        res[name] = ent
    return res


def check(src: str) -> list:
    errs = []
    cls = _classes(src)
    want = {"GpuProductionGroupContext": "GroupContext", "GpuElementModP": "ElementModP"}
    for name, iface in want.items():
        if name not in cls or cls[name][0] != iface:
            errs.append(f"{name} must implement {iface} by delegation")
            continue
        ov = _overrides(cls[name][1])
        members = API[iface]
        for m, ent in ov.items():
            if m in API["Any"]:
                continue
            if m not in members:
                errs.append(f"{name}.{m} overrides no upstream member")
                continue
            ref = members[m]
            if ref["kind"] != ent["kind"]:
                errs.append(f"{name}.{m}: {ent['kind']} vs upstream {ref['kind']}")
            elif ref["kind"] == "val" and ref["type"] != ent["type"]:
                errs.append(f"{name}.{m}: type {ent['type']} vs {ref['type']}")
            elif ref["kind"] == "fun" and (ref["params"] != ent["params"] or ref["returns"] != ent["returns"]):
                errs.append(f"{name}.{m}: ({ent['params']}) -> {ent['returns']} vs ({ref['params']}) -> {ref['returns']}")
        for m, target in API["hot_path"][iface].items():
            if m not in ov:
                errs.append(f"{name}: hot-path member {m} is not overridden")
            elif target + "(" not in ov[m]["expr"]:
                errs.append(f"{name}.{m} does not reach {target}")
            elif members[m].get("returns") == "ElementModP" and not ov[m]["expr"].startswith(("wrap(", "ctx.wrap(")):
                errs.append(f"{name}.{m} returns an unwrapped upstream element")
        # every ElementModP-typed argument is wrapped into a GPU element before the algebra sees it
        for m, ent in ov.items():
            for p, n in zip(ent.get("params", []), ent.get("names", [])):
                if p == "ElementModP" and f"wrap({n})" not in ent["expr"]:
                    errs.append(f"{name}.{m} passes its ElementModP argument {n} on without wrap")
        if iface == "GroupContext":
            for c in ("ONE_MOD_P", "G_MOD_P", "GINV_MOD_P", "G_SQUARED_MOD_P", "binaryToElementModP"):
                if c not in ov or "wrap(" not in ov[c]["expr"]:
                    errs.append(f"{name}.{c} must hand out GPU elements")
    return errs


def test_adapter_matches_the_upstream_members():
    assert check(KT.read_text()) == []


@pytest.mark.parametrize("mutation", ["param", "return", "unwrap", "route", "constant", "delegation", "wrapres",
                                      "accelerate"])
def test_checker_catches_a_broken_adapter(mutation):
    src = KT.read_text()
    rep = {
        "param": ("override infix fun powP(e: ElementModQ)", "override infix fun powP(e: ElementModP)"),
        "return": ("override fun multInv(): ElementModP", "override fun multInv(): ElementModP?"),
        "unwrap": ("ctx.times(this, ctx.wrap(other))", "ctx.times(this, other as GpuElementModP)"),
        "route": ("wrap(defer(Form.fixed(gpu.gTable(), big(e))))", "wrap(base.gPowP(e))"),
        "constant": ("override val G_MOD_P: ElementModP get() = wrap(base.G_MOD_P)",
                     "override val G_MOD_P: ElementModP get() = base.G_MOD_P"),
        "delegation": (": ElementModP by forwarding(cell) {", ": ElementModP {"),
        "wrapres": ("= ctx.wrap(ctx.powP(this, e))", "= ctx.powP(this, e)"),
        "accelerate": ("= ctx.wrap(ctx.accelerate(this))", "= this"),
    }[mutation]
    assert rep[0] in src, "mutation did not apply"
    assert check(src.replace(rep[0], rep[1], 1)) != []


def test_hot_path_natives_exist():
    """The GPU context methods the adapter's algebra submits to: the general per-element job
    (eg_mexp_submit) and its ticket, the per-element tables (g's 16-bit one, acceleratePow's), the
    constant-time switch of a trustee's context, and the batch product."""
    java = (KT.parent.parent.parent.parent / "java" / "electionguard" / "gpu" / "GpuGroupContext.java").read_text()
    for sig, native in (("public long submitJob(", "EgHip.mexpSubmit"),
                        ("public byte[] waitJob(long ticket)", "EgHip.ticketWait"),
                        ("public Table table(ElementModP base, int windowBits)", "EgHip.fixedBaseCreate"),
                        ("public synchronized Table gTable()", "table(group.getG_MOD_P(), 16)"),
                        ("public void setConstantTime(boolean on)", "EgHip.setCtPow"),
                        ("public ElementModP prodP(List<ElementModP> xs)", "EgHip.prodReduce")):
        i = java.index(sig)
        assert native in java[i:java.index("\n  }", i)], sig
    kt = KT.read_text()
    assert "fun trustee(" in kt and "setConstantTime(true)" in kt  # a trustee's context is constant-time
