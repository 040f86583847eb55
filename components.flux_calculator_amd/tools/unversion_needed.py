#!/usr/bin/env python3
"""Rewrite DT_NEEDED 'libamdhip64.so.7' -> 'libamdhip64.so' in an ELF64 shared object.

PyTorch-ROCm ships its own HIP runtime as torch/lib/libamdhip64.so (no SONAME) and its
libraries load it by the unversioned name.  With the unversioned DT_NEEDED, libfcx binds
to whichever HIP runtime the process already has (torch's, or /opt/rocm's when libfcx is
loaded first, which torch then reuses): exactly one HIP runtime per process, so device
pointers, streams and events are shared objects.  The in-place rewrite only shortens a
string in .dynstr (the same thing `patchelf --replace-needed` does for a shorter name).
"""
import struct
import sys

OLD, NEW = b"libamdhip64.so.7\0", b"libamdhip64.so\0"


def main(path):
    data = bytearray(open(path, "rb").read())
    assert data[:4] == b"\x7fELF" and data[4] == 2, "ELF64 expected"
    e_shoff, = struct.unpack_from("<Q", data, 0x28)
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, e_shoff + i * e_shentsize) for i in range(e_shnum)]
    shstr = secs[e_shstrndx]
    names = lambda off: data[shstr[4] + off: data.index(b"\0", shstr[4] + off)].decode()  # noqa: E731
    dynstr = next(s for s in secs if names(s[0]) == ".dynstr")
    lo, hi = dynstr[4], dynstr[4] + dynstr[5]
    at = data.find(OLD, lo, hi)
    if at < 0:
        if data.find(NEW, lo, hi) >= 0:
            return 0  # already rewritten
        raise SystemExit(f"{path}: {OLD!r} not in .dynstr")
    data[at: at + len(OLD)] = NEW + b"\0" * (len(OLD) - len(NEW))
    open(path, "wb").write(bytes(data))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
