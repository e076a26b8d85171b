"""The Rust binding documented in INTEGRATION.md (the reference-side `rtw-sys`
stub -- not compilable here, no Rust toolchain) against the C header: the
`#[repr(C)]` structs must have the C structs' fields in the same order at the
same offsets with the same sizes, and the `extern "C"` block must declare
exactly the entry points of include/rtw.h.  Three views are compared: the
Rust field lists (parsed from INTEGRATION.md, laid out by the repr(C) rules),
gcc's offsetof/sizeof on include/rtw.h, and the ctypes mirror (_capi.py)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from ray_tracing_weekend_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRUCTS = ("rtw_camera_builder", "rtw_camera", "rtw_scene", "rtw_stats")
# Rust type -> (size, align) on x86-64 / aarch64 (repr(C) == the C ABI)
PRIM = {"i32": (4, 4), "u32": (4, 4), "f32": (4, 4), "u8": (1, 1), "i64": (8, 8), "u64": (8, 8), "f64": (8, 8),
        "usize": (8, 8), "c_int": (4, 4)}


def _rust_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.findall(r"```rust\n(.*?)```", text, re.S)


def _rust_struct(name):
    for block in _rust_blocks():
        m = re.search(r"#\[repr\(C\)\][^\n]*\n\s*pub struct " + name + r" \{(.*?)\n\}", block, re.S)
        if m:
            body = re.sub(r"//[^\n]*", "", m.group(1))
            return re.findall(r"pub (\w+): ([^,\n]+?)\s*(?:,|$)", body, re.M)
    raise AssertionError(f"struct {name} not found in INTEGRATION.md")


def _rust_type(t):
    t = t.strip()
    if t.startswith("*const") or t.startswith("*mut"):
        return 8, 8
    m = re.fullmatch(r"\[(\w+); (\d+)\]", t)
    if m:
        s, a = PRIM[m.group(1)]
        return s * int(m.group(2)), a
    return PRIM[t]


def _rust_layout(name):
    off, out, align = 0, [], 1
    for field, t in _rust_struct(name):
        s, a = _rust_type(t)
        off = (off + a - 1) // a * a
        out.append((field, off, s))
        off += s
        align = max(align, a)
    return out, (off + align - 1) // align * align


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    """offsetof / sizeof of every ctypes-mirrored field, from gcc on rtw.h."""
    d = tmp_path_factory.mktemp("layout")
    lines = ["#include <stddef.h>", "#include <stdio.h>", '#include "rtw.h"', "int main(void) {"]
    for name in STRUCTS:
        ct = getattr(_capi, name)
        lines.append(f'printf("{name} sizeof %zu\\n", sizeof({name}));')
        for field, _ in ct._fields_:
            lines.append(f'printf("{name} {field} %zu %zu\\n", offsetof({name}, {field}), '
                         f"sizeof((({name} *)0)->{field}));")
    lines.append("return 0; }")
    src = d / "probe.c"
    src.write_text("\n".join(lines))
    exe = d / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        parts = line.split()
        if parts[1] == "sizeof":
            out[(parts[0], None)] = int(parts[2])
        else:
            out[(parts[0], parts[1])] = (int(parts[2]), int(parts[3]))
    return out


@pytest.mark.parametrize("name", STRUCTS)
def test_rust_struct_matches_c_header(name, c_layout):
    fields, size = _rust_layout(name)
    ct = getattr(_capi, name)
    assert [f for f, _, _ in fields] == [f for f, _ in ct._fields_], "field names / order differ from rtw.h"
    for field, off, sz in fields:
        assert c_layout[(name, field)] == (off, sz), (name, field, c_layout[(name, field)], (off, sz))
    assert c_layout[(name, None)] == size


@pytest.mark.parametrize("name", STRUCTS)
def test_ctypes_mirror_matches_c_header(name, c_layout):
    ct = getattr(_capi, name)
    for field, ftype in ct._fields_:
        assert c_layout[(name, field)] == (getattr(ct, field).offset, C.sizeof(ftype)), (name, field)
    assert c_layout[(name, None)] == C.sizeof(ct)


def test_rust_extern_block_declares_every_entry_point():
    header = open(os.path.join(ROOT, "include", "rtw.h")).read()
    c_fns = set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(rtw_\w+)\s*\(", header, re.M))
    rust = set()
    for block in _rust_blocks():
        m = re.search(r'extern "C" \{(.*?)\n\}', block, re.S)
        if m:
            rust |= set(re.findall(r"pub fn (rtw_\w+)\(", m.group(1)))
    assert rust == c_fns == {p[0] for p in _capi.PROTOTYPES}, (rust ^ c_fns, c_fns ^ {p[0] for p in _capi.PROTOTYPES})
    m = re.search(r"RTW_ABI_VERSION: c_int = (\d+);", "\n".join(_rust_blocks()))
    assert m and int(m.group(1)) == _capi.ABI_VERSION


def test_scene_soa_fills_every_rtw_scene_field():
    """SceneSoA::to_c in INTEGRATION.md sets every field of rtw_scene (a
    struct literal that missed one would not compile)."""
    block = next(b for b in _rust_blocks() if "fn to_c(&self) -> rtw_sys::rtw_scene" in b)
    lit = block[block.index("rtw_sys::rtw_scene {", block.index("fn to_c(&self) -> rtw_sys::rtw_scene")):]
    lit = lit[: lit.index("\n        }")]
    set_fields = set(re.findall(r"(\w+):", lit))
    assert {f for f, _ in _capi.rtw_scene._fields_} <= set_fields
    cam = block[block.index("rtw_sys::rtw_camera {"):]
    cam = cam[: cam.index("\n        }")]
    assert {f for f, _ in _capi.rtw_camera._fields_} <= set(re.findall(r"(\w+):", cam))
