"""Debug: raise one kernel's VGPR allocation in a built
libmcdc.so WITHOUT changing its code.

The kernel descriptor (``<kernel>.kd``, 64 bytes) holds the granulated VGPR
count the hardware allocates (COMPUTE_PGM_RSRC1[5:0], granule 8 on gfx950).
This tool reads the descriptor from the device code object hipcc left with
``-save-temps`` for the same translation unit and flags, finds that exact
64-byte pattern in the shared library's (uncompressed) offload bundle, and
rewrites the granule field.  Only raising is allowed: the kernel's
instructions, register assignment and schedule stay byte-identical, only the
allocation grows past the registers it uses, so it separates "the allocation
ends at the last register used" from "this particular code".

    python tools/dbg/kd_patch.py LIB.so CODE_OBJECT.out KERNEL_SUBSTR NEW_VGPRS OUT.so [NEW_ACCUM_OFFSET]

NEW_ACCUM_OFFSET (optional) also moves COMPUTE_PGM_RSRC3.ACCUM_OFFSET (the
first AGPR of the unified register file; the kernels here use no AGPRs) --
only upwards and never past the new allocation, so the registers the code
names stay architectural VGPRs.
"""
import os
import struct
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from mapache_amd import devaudit as A  # noqa: E402


def main(lib, co, ksub, new_vgprs, out, new_acc=None):
    import re
    import subprocess
    syms = subprocess.run([f"{A.LLVM}/llvm-readelf", "-sW", co], capture_output=True, text=True, check=True).stdout
    secs = subprocess.run([f"{A.LLVM}/llvm-readelf", "-SW", co], capture_output=True, text=True, check=True).stdout
    cdata = open(co, "rb").read()
    sec = {}
    for m in re.finditer(r"\[\s*(\d+)\]\s+(\S+)\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)", secs):
        sec[int(m.group(1))] = (int(m.group(3), 16), int(m.group(4), 16))
    hits = []
    for m in re.finditer(r"\s([0-9a-f]{16})\s+64\s+OBJECT\s+\S+\s+\S+\s+(\d+)\s+(\S+)\.kd$", syms, re.M):
        if ksub in m.group(3):
            addr, ndx = int(m.group(1), 16), int(m.group(2))
            saddr, soff = sec[ndx]
            hits.append((m.group(3), cdata[soff + addr - saddr: soff + addr - saddr + 64]))
    hits = list({h[0]: h for h in hits}.values())  # .symtab and .dynsym both list it
    if len(hits) != 1:
        raise SystemExit(f"{len(hits)} kernels match {ksub!r}: {[h[0] for h in hits]}")
    name, kd = hits[0]
    rsrc1 = struct.unpack_from("<I", kd, 48)[0]
    g_old = rsrc1 & 0x3F
    g_new = new_vgprs // 8 - 1
    if new_vgprs % 8 or g_new <= g_old or g_new > 63:
        raise SystemExit(f"refusing: {name} allocates {(g_old + 1) * 8}, asked {new_vgprs} (raise only, granule 8)")
    data = bytearray(open(lib, "rb").read())
    pos = data.find(kd)
    if pos < 0 or data.find(kd, pos + 1) >= 0:
        raise SystemExit("descriptor not found exactly once in the library (compressed bundle or different build?)")
    struct.pack_into("<I", data, pos + 48, (rsrc1 & ~0x3F) | g_new)
    msg = ""
    if new_acc is not None:
        rsrc3 = struct.unpack_from("<I", kd, 44)[0]
        a_old = ((rsrc3 & 0x3F) + 1) * 4
        if new_acc % 4 or new_acc < a_old or new_acc > new_vgprs:
            raise SystemExit(f"refusing accum_offset {new_acc} (now {a_old}, allocation {new_vgprs})")
        struct.pack_into("<I", data, pos + 44, (rsrc3 & ~0x3F) | (new_acc // 4 - 1))
        msg = f", accum_offset {a_old} -> {new_acc}"
    open(out, "wb").write(bytes(data))
    print(f"{name}: VGPR allocation {(g_old + 1) * 8} -> {new_vgprs}{msg} at file offset {pos:#x}; wrote {out}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5],
         int(sys.argv[6]) if len(sys.argv) > 6 else None)
