"""The reference-side binding helpers (examples/ref_binding/icw_ref_bind.c) read only fields the
reference's types have, and the constants they pass through unchanged have the same values on both
sides.  The helpers compile only inside the reference tree (in_cwave.h needs <windows.h>), so this
CPU test checks them against the reference headers' text: every `var->a.b.c` path resolves through
the typedefs of in_cwave.h, hblpf.h, sound_render.h and cwave.h, and every `out->` / `d->` path
through include/icw.h."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/src")
BIND = ROOT / "examples" / "ref_binding" / "icw_ref_bind.c"

pytestmark = pytest.mark.skipif(not (REF / "in_cwave.h").exists(), reason="reference tree absent")

_SKIP = {"volatile", "const", "struct", "union", "unsigned", "signed"}


def _strip_comments(s):
    return re.sub(r"/\*.*?\*/|//[^\n]*", "", s, flags=re.S)


def typedefs(paths):
    """{type name: {field: field type}} for every `typedef struct|union [tag] { ... } NAME;`"""
    out = {}
    for p in paths:
        text = _strip_comments(Path(p).read_text(errors="replace"))
        for m in re.finditer(r"typedef\s+(?:struct|union)\s*(\w*)\s*\{(.*?)\}\s*(\w+)\s*;", text, re.S):
            tag, body, name = m.groups()
            fields = {}
            for decl in body.split(";"):
                parts = re.sub(r"\[[^\]]*\]", "", decl).split(",")   # "T a, b, c;"
                toks = [t for t in re.findall(r"[A-Za-z_]\w*", parts[0]) if t not in _SKIP]
                if not toks:
                    continue
                ftype = toks[-2] if len(toks) >= 2 else "unsigned"      # "unsigned x;"
                fields[toks[-1]] = ftype
                for extra in parts[1:]:
                    names = re.findall(r"[A-Za-z_]\w*", extra)
                    if names:
                        fields[names[-1]] = ftype
            out[name] = fields
            if tag:
                out[tag] = fields
        for m in re.finditer(r"typedef\s+(\w+)\s+(\w+)\s*;", text):    # typedef HCWAVE_V2 HCWAVE;
            if m.group(1) in out:
                out[m.group(2)] = out[m.group(1)]
    return out


def paths_of(var, text):
    return sorted(set(re.findall(rf"\b{var}->(\w+(?:\.\w+)*)", text)))


def resolve(types, root, path):
    t = root
    for f in path.split("."):
        assert t in types, f"{root}.{path}: {t} is not a struct the headers define"
        assert f in types[t], f"{root}.{path}: {t} has no field {f}"
        t = types[t][f]
    return t


def test_reference_fields_exist():
    ref = typedefs([REF / "in_cwave.h", REF / "hblpf.h", REF / "sound_render.h", REF / "cwave.h"])
    text = _strip_comments(BIND.read_text())
    seen = 0
    for var, root in (("cfg", "IN_CWAVE_CFG"), ("s", "NODE_DSP"), ("head", "NODE_DSP"), ("xr", "XWAVE_READER")):
        for p in paths_of(var, text):
            resolve(ref, root, p)
            seen += 1
    assert seen >= 40                      # every node field, the config fields, the reader fields


def test_icw_fields_exist():
    icw = typedefs([ROOT / "include" / "icw.h"])
    text = _strip_comments(BIND.read_text())
    for var, root in (("out", "icw_config"), ("d", "icw_node")):
        ps = paths_of(var, text)
        assert ps
        for p in ps:
            resolve(icw, root, p)


def _defines(path):
    d = {}
    for m in re.finditer(r"#define\s+(\w+)\s+\(?\s*(0x[0-9A-Fa-f]+|-?\d+)U?\s*\)?", Path(path).read_text(errors="replace")):
        d[m.group(1)] = int(m.group(2), 0)
    return d


def test_pass_through_constants_agree():
    ref = {**_defines(REF / "in_cwave.h"), **_defines(REF / "cwave.h"), **_defines(REF / "sound_render.h")}
    icw = _defines(ROOT / "include" / "icw.h")
    pairs = [("MODE_MASTER", "ICW_MODE_MASTER"), ("MODE_SHIFT", "ICW_MODE_SHIFT"),
             ("MODE_PM", "ICW_MODE_PM"), ("MODE_MIX", "ICW_MODE_MIX"),
             ("S_ADD_REIM", "ICW_S_ADD_REIM"), ("S_SUB_REIM", "ICW_S_SUB_REIM"), ("S_RE", "ICW_S_RE"),
             ("S_IM", "ICW_S_IM"), ("XCH_NORMAL", "ICW_XCH_NORMAL"), ("XCH_SWAP", "ICW_XCH_SWAP"),
             ("XCH_LEFTONLY", "ICW_XCH_LEFTONLY"), ("XCH_RIGHTONLY", "ICW_XCH_RIGHTONLY"),
             ("XCH_MIXLR", "ICW_XCH_MIXLR"), ("HRW_FMT_UINT8", "ICW_FMT_U8"), ("HRW_FMT_INT16", "ICW_FMT_I16"),
             ("HRW_FMT_INT24", "ICW_FMT_I24"), ("HRW_FMT_INT32", "ICW_FMT_I32"), ("HRW_FMT_FLOAT32", "ICW_FMT_F32")]
    for r, i in pairs:
        assert ref[r] == icw[i], (r, i)
    # CWAVE: ICW_FMT_CW_* = ICW_FMT_CW_F64 + HCW_FMT_PCM_*  (icw_fmt_from_reader)
    for r, i in (("HCW_FMT_PCM_DBL64", "ICW_FMT_CW_F64"), ("HCW_FMT_PCM_INT16", "ICW_FMT_CW_I16"),
                 ("HCW_FMT_PCM_INT16_FLT32", "ICW_FMT_CW_I16_F32"), ("HCW_FMT_PCM_FLT32", "ICW_FMT_CW_F32")):
        assert icw["ICW_FMT_CW_F64"] + ref[r] == icw[i], (r, i)
    # the render seeds of mod_context_init (in_cwave.c:69-70)
    init = (REF / "in_cwave.c").read_text(errors="replace")
    seeds = [int(x, 16) for x in re.findall(r"sound_render_init\([^;]*?(0x[0-9A-Fa-f]+)", init)]
    assert seeds == [icw["ICW_SEED_LEFT"], icw["ICW_SEED_RIGHT"]]
