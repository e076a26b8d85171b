"""Code-object identity of the gfx950 kernels inside librtw.so.

Measurement infrastructure (bench.py, tools/pmc_summary.py): a rocprofv3 PMC
profile committed under profiles/ is only valid for the machine code it was
taken on, so every profile records the ISA hash of the kernel it measured and
bench.py attaches its counters to a line only when the kernel that ran has the
same hash in the library that is loaded now.

The hash covers the kernel's machine code (its FUNC symbol in the gfx950 code
object) and its 64-B kernel descriptor (`<name>.kd`: VGPR / SGPR / LDS /
scratch settings) with the code-entry offset zeroed (it shifts when another
kernel of the same code object changes size).  Pure Python: the library's `.hip_fatbin` section holds
clang offload bundles ("__CLANG_OFFLOAD_BUNDLE__", one per HIP translation
unit), each with an amdgcn ELF code object per target.
"""
from __future__ import annotations

import hashlib
import os
import struct

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "librtw.so")


def _elf_sections(blob: bytes):
    """(name, type, addr, offset, size, link) of every section of an ELF64."""
    if blob[:4] != b"\x7fELF" or blob[4] != 2:
        raise ValueError("not an ELF64 object")
    shoff, = struct.unpack_from("<Q", blob, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", blob, 0x3A)
    raw = []
    for k in range(shnum):
        name, typ, _flags, addr, off, size, link = struct.unpack_from("<IIQQQQI", blob, shoff + k * shentsize)
        raw.append((name, typ, addr, off, size, link))
    stroff = raw[shstrndx][3]

    def cstr(base, at):
        end = blob.index(b"\0", base + at)
        return blob[base + at:end].decode()
    return [(cstr(stroff, n), t, a, o, s, l) for (n, t, a, o, s, l) in raw]


def gfx950_code_objects(lib: str = LIB):
    """The gfx950 code objects bundled in `lib` (bytes each)."""
    data = open(lib, "rb").read()
    secs = {s[0]: s for s in _elf_sections(data)}
    if ".hip_fatbin" not in secs:
        raise ValueError(f"{lib}: no .hip_fatbin section")
    _, _, _, off, size, _ = secs[".hip_fatbin"]
    fat = data[off:off + size]
    out = []
    pos = fat.find(_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + len(_MAGIC))
        q = pos + len(_MAGIC) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" in triple and esize:
                out.append(fat[pos + eoff:pos + eoff + esize])
        pos = fat.find(_MAGIC, pos + 1)
    return out


def _symbols(co: bytes):
    secs = _elf_sections(co)
    for (name, typ, addr, off, size, link) in secs:
        if typ != 2:   # SHT_SYMTAB
            continue
        stroff = secs[link][3]
        for k in range(size // 24):
            st_name, st_info, _o, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", co, off + k * 24)
            end = co.index(b"\0", stroff + st_name)
            yield co[stroff + st_name:end].decode(), st_info & 15, st_shndx, st_value, st_size, secs


def kernel_bytes(co: bytes):
    """{kernel symbol: machine code + kernel descriptor} of one code object."""
    code, kd = {}, {}
    for name, typ, shndx, value, size, secs in _symbols(co):
        if shndx == 0 or shndx >= len(secs) or size == 0:
            continue
        _n, _t, addr, off, _s, _l = secs[shndx]
        body = co[off + value - addr:off + value - addr + size]
        if typ == 2:            # STT_FUNC
            code[name] = body
        elif name.endswith(".kd"):
            # bytes 16..23: kernel_code_entry_byte_offset, the distance from
            # the descriptor to the code -- it moves whenever another kernel of
            # the same code object changes size, the machine code does not
            kd[name[:-3]] = body[:16] + bytes(8) + body[24:] if len(body) >= 24 else body
    return {k: v + kd.get(k, b"") for k, v in code.items()}


def render_kernel_symbol(dtype: str, world: int, opts: int) -> str:
    """Itanium name of rtw::dev::render_kernel<R, kWorld, kOpt>(KParams<R>)."""
    r = {"f32": "f", "float": "f", "f64": "d", "double": "d"}[dtype]
    return f"_ZN3rtw3dev13render_kernelI{r}Li{int(world)}ELi{int(opts)}EEEvNS_7KParamsIT_EE"


def render_kernel_name(dtype: str, world: int, opts: int) -> str:
    """rocprofv3's (demangled) name of the same kernel."""
    r = {"f32": "float", "float": "float", "f64": "double", "double": "double"}[dtype]
    return f"void rtw::dev::render_kernel<{r}, {int(world)}, {int(opts)}>(rtw::KParams<{r}>)"


_cache: dict = {}


def kernel_isa_sha(symbol: str, lib: str = LIB) -> str | None:
    """sha256 (first 16 hex digits) of the kernel's machine code + descriptor
    in `lib`, or None if no gfx950 code object has that kernel."""
    key = (lib, os.path.getmtime(lib))
    if key not in _cache:
        table = {}
        for co in gfx950_code_objects(lib):
            table.update(kernel_bytes(co))
        _cache.clear()
        _cache[key] = {k: hashlib.sha256(v).hexdigest()[:16] for k, v in table.items()}
    return _cache[key].get(symbol)


def demangled_to_symbol(name: str) -> str | None:
    """rocprofv3's `void rtw::dev::render_kernel<float, 5, 16>(...)` -> symbol."""
    import re
    m = re.match(r"void rtw::dev::render_kernel<(float|double), (\d+), (\d+)>", name)
    return render_kernel_symbol(m.group(1), int(m.group(2)), int(m.group(3))) if m else None
