"""Per-kernel register / spill / scratch metadata of the built gfx950 code
objects, read straight from a linked library's (or object's) .hip_fatbin
section: clang offload bundles -> the gfx950 ELF -> its AMDGPU metadata note
(msgpack).  No recompilation, no GPU.

    python3 tools/kernel_meta.py [beta-sgp_amd/libbsgp.so]

prints one line per kernel: VGPRs, AGPRs, VGPR spills, SGPR spills, private
segment bytes (scratch per lane), LDS bytes.  tests/test_regbudget.py holds the
allow-list these must stay within.
"""
import struct
import sys

import msgpack

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(elf, name):
    """Bytes of section `name` of a 64-bit little-endian ELF image."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    def hdr(i):
        return struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize)
    strtab = hdr(shstrndx)
    for i in range(shnum):
        h = hdr(i)
        nm = elf[strtab[4] + h[0]:elf.index(b"\0", strtab[4] + h[0])].decode()
        if nm == name:
            return elf[h[4]:h[4] + h[5]]
    return None


def _notes(elf):
    """(name, type, desc) of every note of the ELF's .note section."""
    sec = _section(elf, ".note")
    out, o = [], 0
    while sec is not None and o + 12 <= len(sec):
        namesz, descsz, typ = struct.unpack_from("<III", sec, o)
        o += 12
        name = sec[o:o + namesz].rstrip(b"\0").decode()
        o += (namesz + 3) & ~3
        out.append((name, typ, sec[o:o + descsz]))
        o += (descsz + 3) & ~3
    return out


def code_objects(path, arch="gfx950"):
    """Every `arch` code object ELF in the file's offload bundles."""
    data = open(path, "rb").read()
    fb = _section(data, ".hip_fatbin") if data[:4] == b"\x7fELF" else data
    if fb is None:
        return []
    objs, pos = [], fb.find(_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fb, pos + len(_MAGIC))
        o = pos + len(_MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fb, o)
            triple = fb[o + 24:o + 24 + tlen].decode()
            o += 24 + tlen
            if triple.endswith(arch):
                objs.append(fb[pos + off:pos + off + size])
        pos = fb.find(_MAGIC, pos + 1)
    return objs


def kernels(path, arch="gfx950"):
    """{kernel symbol: metadata dict} over every code object of the file."""
    res = {}
    for co in code_objects(path, arch):
        for name, typ, desc in _notes(co):
            if name != "AMDGPU" or typ != 32:  # NT_AMDGPU_METADATA
                continue
            meta = msgpack.unpackb(desc, raw=False)
            for k in meta.get("amdhsa.kernels", []):
                res[k[".name"]] = {
                    "vgpr": k.get(".vgpr_count"),
                    "agpr": k.get(".agpr_count", 0),
                    "vgpr_spill": k.get(".vgpr_spill_count", 0),
                    "sgpr_spill": k.get(".sgpr_spill_count", 0),
                    "private": k.get(".private_segment_fixed_size", 0),
                    "lds": k.get(".group_segment_fixed_size", 0),
                    "dyn_stack": k.get(".uses_dynamic_stack", False),
                }
    return res


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else "beta-sgp_amd/libbsgp.so"
    for name, m in sorted(kernels(lib).items()):
        print(f"{name[:90]:90s} vgpr={m['vgpr']:3d} spill={m['vgpr_spill']:3d} "
              f"sspill={m['sgpr_spill']:3d} scratch={m['private']:4d} dyn={int(m['dyn_stack'])}")
