"""The gfx950 machine code of individual kernels in libfedagg.so, as a stable key for measurements.

hipcc embeds the device code as a clang offload bundle in the host library's ``.hip_fatbin`` section;
the gfx950 entry is an AMDGPU ELF whose kernels are STT_FUNC symbols (their instructions in
``.text``) plus ``<kernel>.kd`` descriptors (register counts, LDS, launch properties) in
``.rodata``. A measurement of one kernel — the rocprofv3 PMC traffic in profiles/pmc_traffic.json —
stays valid exactly as long as those bytes are unchanged: edits to other kernels, the build
directory (hipcc's ``__hip_cuid_<hash>`` follows the build paths) or host code do not touch them.
``kernel_sha`` hashes them; bench.py compares it with the sha recorded when the PMC run was made.
"""
import hashlib
import shutil
import struct
import subprocess

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    """[(name, type, addr, offset, size, link)] of an ELF64 little-endian image."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not an ELF64 little-endian image")
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    raw = [struct.unpack_from("<IIQQQQII", elf, shoff + i * shentsize) for i in range(shnum)]
    stroff = raw[shstrndx][4]

    def name(n):
        end = elf.index(b"\0", stroff + n)
        return elf[stroff + n:end].decode()
    return [(name(n), t, addr, off, size, link) for n, t, _flags, addr, off, size, link, _info in raw]


def gfx950_code_object(lib_path, arch="gfx950"):
    """The ``arch`` device ELF inside a HIP host library (uncompressed offload bundle)."""
    with open(lib_path, "rb") as f:
        data = f.read()
    secs = _sections(data)
    fat = next((s for s in secs if s[0] == ".hip_fatbin"), None)
    if fat is None:
        raise ValueError(f"{lib_path}: no .hip_fatbin section")
    base = fat[3]
    if data[base:base + len(_BUNDLE_MAGIC)] != _BUNDLE_MAGIC:
        raise ValueError(f"{lib_path}: .hip_fatbin is not an uncompressed offload bundle")
    n = struct.unpack_from("<Q", data, base + 24)[0]
    p = base + 32
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", data, p)
        triple = data[p + 24:p + 24 + tlen].decode()
        p += 24 + tlen
        if triple.endswith(arch) or f"--{arch}" in triple:
            return data[base + off:base + off + size]
    raise ValueError(f"{lib_path}: no {arch} code object in the bundle")


def symbols(co):
    """{name: bytes} of every defined FUNC / OBJECT symbol of a device ELF (code and .kd)."""
    secs = _sections(co)
    symtab = next((s for s in secs if s[1] == 2), None)   # SHT_SYMTAB
    if symtab is None:
        raise ValueError("code object has no symbol table")
    _, _, _, soff, ssize, link = symtab
    strtab_off = secs[link][3]
    out = {}
    for k in range(ssize // 24):
        st_name, st_info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", co, soff + 24 * k)
        if st_info & 0xF not in (1, 2) or shndx == 0 or shndx >= len(secs) or size == 0:   # OBJECT, FUNC
            continue
        end = co.index(b"\0", strtab_off + st_name)
        name = co[strtab_off + st_name:end].decode()
        _, _, addr, off, _, _ = secs[shndx]
        out[name] = co[off + (value - addr):off + (value - addr) + size]
    return out


def demangle(names):
    """Demangled names (llvm-cxxfilt / c++filt), in order; the input where no tool is found."""
    tool = shutil.which("llvm-cxxfilt") or "/opt/rocm/lib/llvm/bin/llvm-cxxfilt"
    if not shutil.which(tool):
        tool = shutil.which("c++filt")
    if not tool:
        return list(names)
    res = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True, check=True)
    return res.stdout.splitlines()


def _short(demangled):
    """A demangled kernel as rocprofv3 names it: no return type, no anonymous-namespace qualifiers."""
    d = demangled.replace("(anonymous namespace)::", "")
    return d[5:] if d.startswith("void ") else d


def kernels_matching(lib_path, kernel):
    """Mangled names of the kernels whose demangled name contains ``kernel`` (a string, or a list of
    strings that must all appear — rocprofv3's Kernel_Name matching in tools/pmc_traffic.py), in
    the full or the :func:`_short` form, with their ``.kd`` descriptors; sorted."""
    parts = [kernel] if isinstance(kernel, str) else list(kernel)
    syms = symbols(gfx950_code_object(lib_path))
    funcs = sorted(n for n in syms if not n.endswith(".kd"))
    picked = [m for m, d in zip(funcs, demangle(funcs))
              if all(p in d for p in parts) or all(p in _short(d) for p in parts)]
    return sorted(picked + [m + ".kd" for m in picked if m + ".kd" in syms])


# amd_kernel_code_t / kernel descriptor: bytes 16-23 hold kernel_code_entry_byte_offset, the distance
# from the descriptor to the kernel's code — where the linker placed the two, not the kernel (adding a
# kernel elsewhere in the library moves it). The rest (segment sizes, register and mode settings)
# describe the kernel and stay in the key.
_KD_ENTRY_OFFSET = slice(16, 24)


def _keyed(name, data):
    if name.endswith(".kd") and len(data) >= _KD_ENTRY_OFFSET.stop:
        data = data[:_KD_ENTRY_OFFSET.start] + bytes(8) + data[_KD_ENTRY_OFFSET.stop:]
    return data


def kernel_sha(lib_path, names):
    """sha256 (16 hex) over the machine code and descriptors of ``names`` (mangled, as
    :func:`kernels_matching` lists them) in the gfx950 code object — the descriptors without their
    layout-dependent code offset; None if one is missing."""
    syms = symbols(gfx950_code_object(lib_path))
    h = hashlib.sha256()
    for n in sorted(names):
        if n not in syms:
            return None
        h.update(n.encode() + b"\0" + _keyed(n, syms[n]))
    return h.hexdigest()[:16]
