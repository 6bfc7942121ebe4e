"""Identity of the device code a profile belongs to.

PMC summaries (tools/profile_summary.py) are stamped with, and bench.py
compares, the sha256 of libptgpu.so's `.hip_fatbin` section: the gfx950 code
objects of every kernel.  A host-only change (API, loader, statistics) leaves
it unchanged, so committed counter summaries stay valid across such changes;
any change to a kernel changes it.  The whole file's sha256 is kept beside it."""
import hashlib
import struct


def section_bytes(path: str, name: str) -> bytes:
    """Bytes of ELF64 section `name` (little-endian shared object)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise ValueError(f"{path}: not an ELF64 file")
    shoff = struct.unpack_from("<Q", data, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def hdr(i):
        # sh_name, sh_type, sh_flags, sh_addr, sh_offset, sh_size
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)

    stro, strs = hdr(shstrndx)[4], hdr(shstrndx)[5]
    names = data[stro:stro + strs]
    for i in range(shnum):
        h = hdr(i)
        end = names.index(b"\0", h[0])
        if names[h[0]:end].decode() == name:
            return data[h[4]:h[4] + h[5]]
    raise KeyError(f"{path}: no section {name}")


def kernel_sha256(path: str) -> str:
    return hashlib.sha256(section_bytes(path, ".hip_fatbin")).hexdigest()


def file_sha256(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()
