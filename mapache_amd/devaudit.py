"""Static audit of the device code of libmcdc, run by build.py on
every build.

For every kernel (and every non-inlined device function) in a hipcc
``-save-temps`` device assembly file (``*-hip-amdgcn-amd-amdhsa-gfx950.s``) it
reports:

* ``next_free_vgpr`` / ``accum_offset`` from the ``.amdhsa_kernel`` block and
  the highest VGPR index any instruction names (register tuples included);
* whether that top register is ever the destination of a memory load (VMEM or
  LDS), i.e. a register whose value arrives asynchronously;
* **waitcnt coverage**: a data-flow pass over the control-flow graph that tracks
  every outstanding load (``vmcnt`` in issue order; ``lgkmcnt`` in issue order
  for LDS, out of order once a scalar load is pending) with its destination
  registers, retires them at each ``s_waitcnt``, and flags any instruction that
  names a register (as source or destination) whose load is not yet guaranteed
  complete on some path.

Given the device code object (``.out`` / ``.hsaco``) it also decodes every
kernel descriptor: the granulated VGPR count of COMPUTE_PGM_RSRC1 and the
ACCUM_OFFSET of COMPUTE_PGM_RSRC3 (gfx90a+ unified register file), so the
allocation the hardware is told can be compared with the registers used.

    python -m mapache_amd.devaudit DIR_WITH_SAVE_TEMPS [--kernel SUBSTR] [--hazards]
"""
from __future__ import annotations

import argparse
import os
import re
import struct
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"

_VRANGE = re.compile(r"\b([va])\[(\d+):(\d+)\]")
_VONE = re.compile(r"\b([va])(\d+)\b")
_WAIT = re.compile(r"(vmcnt|lgkmcnt|expcnt)\((\d+)\)")
QMAX = 64  # outstanding entries tracked per counter (beyond: the oldest are dropped as retired-unknown)


def regs_of(text: str):
    """VGPR (v) and AGPR (a, offset by 1000) indices named in an operand string."""
    out = set()
    s = _VRANGE.sub(lambda m: out.update(range(int(m.group(2)) + (1000 if m.group(1) == "a" else 0),
                                               int(m.group(3)) + 1 + (1000 if m.group(1) == "a" else 0))) or " ",
                    text)
    for kind, n in _VONE.findall(s):
        out.add(int(n) + (1000 if kind == "a" else 0))
    return out


def split_units(asm: str):
    """{symbol: [lines]} for every function body (kernels and device functions)."""
    units = {}
    for m in re.finditer(r"^([._A-Za-z0-9$]+):[^\n]*\n(.*?)^(\.Lfunc_end\d+):", asm, re.S | re.M):
        name = m.group(1)
        if name.startswith(".LBB"):
            continue
        units[name] = m.group(2).split("\n")
    return units


def kernel_fields(asm: str):
    out = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", asm, re.S):
        f = {}
        for key in ("next_free_vgpr", "accum_offset", "next_free_sgpr"):
            mm = re.search(r"\.amdhsa_" + key + r"\s+(\S+)", m.group(2))
            if mm:
                try:
                    f[key] = int(mm.group(1))
                except ValueError:
                    f[key] = mm.group(1)
        out[m.group(1)] = f
    return out


def max_workgroup_sizes(asm: str):
    """{kernel: .max_flat_workgroup_size} from the code object metadata."""
    return {m.group(2): int(m.group(1))
            for m in re.finditer(r"\.max_flat_workgroup_size:\s+(\d+)\s*\n\s*\.name:\s+(\S+)", asm)}


def vgpr_ceiling(wg_size: int) -> int:
    """Most VGPRs per lane a kernel of this workgroup size may allocate and
    still launch: the block's waves spread over the CU's 4 SIMDs, each SIMD
    holding 512 VGPRs per lane, in 8-register granules."""
    waves_per_simd = -(-(-(-wg_size // 64)) // 4)
    return 512 // max(waves_per_simd, 1) // 8 * 8


class Insn:
    __slots__ = ("idx", "op", "args", "text", "label")

    def __init__(self, idx, op, args, text):
        self.idx, self.op, self.args, self.text = idx, op, args, text


def parse(lines):
    """Instructions and label positions of one unit."""
    insns, labels = [], {}
    for ln in lines:
        s = ln.split(";")[0].strip()
        if not s:
            continue
        if s.endswith(":"):
            labels[s[:-1]] = len(insns)
            continue
        if s.startswith("."):
            continue
        parts = s.split(None, 1)
        insns.append(Insn(len(insns), parts[0], parts[1] if len(parts) > 1 else "", s))
    return insns, labels


def classify(op: str, args: str):
    """(counter set, destination registers or None) of a memory instruction, else None."""
    ret = " sc0" in " " + args or " glc" in " " + args
    if op.startswith(("global_load", "buffer_load", "scratch_load")):
        if " lds" in " " + args:  # LDS DMA: no VGPR destination
            return ("vm",), set()
        return ("vm",), regs_of(args.split(",")[0])
    if op.startswith(("global_atomic", "buffer_atomic", "flat_atomic")):
        cnt = ("vm", "lgkm") if op.startswith("flat") else ("vm",)
        return cnt, (regs_of(args.split(",")[0]) if ret else set())
    if op.startswith(("global_store", "buffer_store", "scratch_store")):
        return ("vm",), set()
    if op.startswith("flat_load"):
        return ("vm", "lgkm"), regs_of(args.split(",")[0])
    if op.startswith("flat_store"):
        return ("vm", "lgkm"), set()
    if op.startswith("ds_"):
        rd = (op.startswith(("ds_read", "ds_load", "ds_swizzle", "ds_permute", "ds_bpermute", "ds_consume",
                             "ds_append")) or "_rtn" in op or op.startswith("ds_gws"))
        return ("lds",), (regs_of(args.split(",")[0]) if rd else set())
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_getreg")) and op.startswith("s_"):
        if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime")):
            return ("smem",), set()
    if op.startswith("s_sendmsg"):
        return ("smem",), set()
    return None


class State:
    """Outstanding loads: vm queue (in order), lgkm queue (LDS in order; SMEM
    entries make the queue out of order).  Entries are frozensets of registers
    (LDS/VMEM destinations) plus the issuing instruction index."""

    def __init__(self, vm=(), lgkm=()):
        self.vm = tuple(vm)
        self.lgkm = tuple(lgkm)

    def key(self):
        return (self.vm, self.lgkm)

    @staticmethod
    def merge(a: "State", b: "State") -> "State":
        def mq(x, y):
            n = max(len(x), len(y))
            x = ((None,) * (n - len(x))) + x
            y = ((None,) * (n - len(y))) + y
            out = []
            for p, q in zip(x, y):
                if p is None:
                    out.append(q)
                elif q is None or p == q:
                    out.append(p)
                else:  # union of the two entries (same slot, different paths)
                    out.append(("mix", p[1] | q[1], p[2] or q[2], min(p[3], q[3])))
            return tuple(out[-QMAX:])
        return State(mq(a.vm, b.vm), mq(a.lgkm, b.lgkm))

    def pending_regs(self):
        r = {}
        for e in self.vm + self.lgkm:
            for reg in e[1]:
                r.setdefault(reg, e[3])
        return r


def step(st: State, ins: Insn, hazards=None, unit=""):
    op, args = ins.op, ins.args
    if op == "s_waitcnt":
        vm = lg = None
        for k, v in _WAIT.findall(args):
            if k == "vmcnt":
                vm = int(v)
            elif k == "lgkmcnt":
                lg = int(v)
        if args.strip() == "0":
            vm = lg = 0
        nvm, nlg = st.vm, st.lgkm
        if vm is not None and len(nvm) > vm:
            nvm = nvm[len(nvm) - vm:] if vm else ()
        if lg is not None:
            if lg == 0:
                nlg = ()
            else:
                # LDS entries return in order among themselves; at most lg
                # entries of any kind are outstanding, so every LDS entry older
                # than the lg newest LDS entries is complete.  Scalar loads
                # return out of order: only lgkmcnt(0) retires them.
                lds = [i for i, e in enumerate(nlg) if not e[2]]
                done = set(lds[:max(0, len(lds) - lg)])
                nlg = tuple(e for i, e in enumerate(nlg) if i not in done)
        return State(nvm, nlg)
    if op.startswith("s_swappc"):
        # a call: the callee starts with a full s_waitcnt (checked in audit())
        return State()
    cls = classify(op, args)
    # hazard check: any named register with a load still outstanding
    if hazards is not None:
        named = regs_of(args)
        pend = st.pending_regs()
        bad = named & set(pend)
        if bad:
            # A load whose destination overlaps an older load of the same
            # in-order queue (and whose address registers are complete) is a
            # write-after-write the in-order return already orders: benign.
            kind = "raw"
            if cls is not None and cls[1] and not (bad - cls[1]):
                vm_regs = set().union(*(e[1] for e in st.vm)) if st.vm else set()
                lds_regs = set().union(*(e[1] for e in st.lgkm)) if st.lgkm else set()
                same = vm_regs if "vm" in cls[0] else lds_regs
                other = lds_regs if "vm" in cls[0] else vm_regs
                if bad <= same and not (bad & other):
                    kind = "waw-in-order"
            hazards.append((unit, ins.idx, ins.text, sorted(bad), pend[min(bad)], kind))
    if cls is None:
        return st
    counters, dst = cls
    ent_v = ("ld", frozenset(dst), False, ins.idx)
    vm, lg = st.vm, st.lgkm
    if "vm" in counters:
        vm = (vm + (ent_v,))[-QMAX:]
    if "lgkm" in counters or "lds" in counters:
        lg = (lg + (("ld", frozenset(dst) if "vm" not in counters else frozenset(), False, ins.idx),))[-QMAX:]
    if "smem" in counters:
        lg = (lg + (("sm", frozenset(), True, ins.idx),))[-QMAX:]
    return State(vm, lg)


def cfg(insns, labels):
    """Basic blocks as (start, end) and successors."""
    leaders = {0} | set(labels.values())
    for i, ins in enumerate(insns):
        if ins.op.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc", "s_swappc")) and i + 1 < len(insns):
            leaders.add(i + 1)
    leaders = sorted(x for x in leaders if x < len(insns))
    blocks = []
    for j, s in enumerate(leaders):
        e = leaders[j + 1] if j + 1 < len(leaders) else len(insns)
        blocks.append((s, e))
    start_of = {s: b for b, (s, _) in enumerate(blocks)}
    succ = []
    for b, (s, e) in enumerate(blocks):
        last = insns[e - 1]
        out = []
        if last.op.startswith("s_branch"):
            out.append(start_of[labels[last.args.strip()]])
        elif last.op.startswith("s_cbranch"):
            out.append(start_of[labels[last.args.strip()]])
            if b + 1 < len(blocks):
                out.append(b + 1)
        elif last.op.startswith(("s_endpgm", "s_setpc")):
            pass
        elif b + 1 < len(blocks):
            out.append(b + 1)
        succ.append(out)
    return blocks, succ


def analyse(insns, labels, unit="", entry=State()):
    blocks, succ = cfg(insns, labels)
    inn = {0: entry}
    work = [0]
    it = 0
    while work and it < 200000:
        it += 1
        b = work.pop()
        st = inn[b]
        s, e = blocks[b]
        for i in range(s, e):
            st = step(st, insns[i])
        for t in succ[b]:
            nst = st if t not in inn else State.merge(inn[t], st)
            if t not in inn or nst.key() != inn[t].key():
                inn[t] = nst
                work.append(t)
    hazards = []
    for b, (s, e) in enumerate(blocks):
        if b not in inn:
            continue
        st = inn[b]
        for i in range(s, e):
            st = step(st, insns[i], hazards, unit)
    return hazards


def top_reg_info(insns):
    top, load_dst = -1, set()
    for ins in insns:
        r = {x for x in regs_of(ins.args) if x < 1000}
        if r:
            top = max(top, max(r))
        cls = classify(ins.op, ins.args)
        if cls and cls[1]:
            load_dst |= {x for x in cls[1] if x < 1000}
    return top, load_dst


def descriptors(code_object: str):
    """{kernel: (granulated vgpr field, vgprs allocated, accum_offset)} from the .kd symbols."""
    return {k: v[:3] for k, v in descriptor_bytes(code_object).items()}


def descriptor_bytes(code_object: str):
    """{kernel: (granule field, vgprs allocated, accum_offset, 64 descriptor bytes)}."""
    syms = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", code_object], capture_output=True, text=True,
                          check=True).stdout
    secs = subprocess.run([f"{LLVM}/llvm-readelf", "-SW", code_object], capture_output=True, text=True,
                          check=True).stdout
    data = open(code_object, "rb").read()
    sec = {}
    for m in re.finditer(r"\[\s*(\d+)\]\s+(\S+)\s+\S+\s+([0-9a-f]+)\s+([0-9a-f]+)\s+([0-9a-f]+)", secs):
        sec[int(m.group(1))] = (int(m.group(3), 16), int(m.group(4), 16))
    out = {}
    for m in re.finditer(r"\s([0-9a-f]{16})\s+64\s+OBJECT\s+\S+\s+\S+\s+(\d+)\s+(\S+)\.kd$", syms, re.M):
        addr, ndx, name = int(m.group(1), 16), int(m.group(2)), m.group(3)
        saddr, soff = sec[ndx]
        kd = data[soff + addr - saddr: soff + addr - saddr + 64]
        rsrc3, rsrc1 = struct.unpack_from("<II", kd, 44)
        g = rsrc1 & 0x3F
        acc = ((rsrc3 & 0x3F) + 1) * 4
        out[name] = (g, (g + 1) * 8, acc, bytes(kd))
    return out


def pad_descriptors(lib: str, asm_dir: str, names) -> list:
    """Raise the VGPR allocation of the named kernels by one 8-register granule
    in the linked shared library `lib`, leaving their code untouched (the cure
    DESIGN.md §3a established: the same instructions with one granule more
    allocated never lost a value).  Each kernel's 64-byte descriptor is taken
    from the code objects hipcc left in asm_dir (-save-temps) and must occur in
    the library's uncompressed offload bundle; a byte pattern shared with a
    kernel that is not to be padded is refused.  Returns [(kernel, old, new)]."""
    names = set(names)
    _, o_files = find_files(asm_dir)
    want, other = {}, set()
    for o in o_files:
        for name, (g, alloc, _acc, kd) in descriptor_bytes(o).items():
            if name in names:
                want.setdefault(kd, set()).add(name)
            else:
                other.add(kd)
    data = bytearray(open(lib, "rb").read())
    done = []
    for kd, ks in want.items():
        if kd in other:
            raise RuntimeError(f"descriptor of {sorted(ks)[0]} is shared with a kernel not to be padded")
        rsrc1 = struct.unpack_from("<I", kd, 48)[0]
        g = rsrc1 & 0x3F
        if g + 1 > 63:
            raise RuntimeError(f"{sorted(ks)[0]}: allocation cannot grow past 512 VGPRs")
        new = kd[:48] + struct.pack("<I", (rsrc1 & ~0x3F) | (g + 1)) + kd[52:]
        pos, hits = data.find(kd), 0
        while pos >= 0:
            data[pos:pos + 64] = new
            hits += 1
            pos = data.find(kd, pos + 64)
        if hits == 0:
            raise RuntimeError(f"descriptor of {sorted(ks)[0]} not found in {lib} (compressed bundle?)")
        done += [(k, (g + 1) * 8, (g + 2) * 8) for k in sorted(ks)]
    open(lib, "wb").write(bytes(data))
    return done


def library_allocations(lib: str, asm_dir: str, names):
    """{kernel: VGPRs allocated} for the named kernels as the library's own
    descriptors say (each located by its bytes outside the granule field)."""
    names = set(names)
    data = open(lib, "rb").read()
    _, o_files = find_files(asm_dir)
    out = {}
    for o in o_files:
        for name, (g, alloc, _acc, kd) in descriptor_bytes(o).items():
            if name not in names:
                continue
            for cand in range(64):
                rsrc1 = struct.unpack_from("<I", kd, 48)[0]
                probe = kd[:48] + struct.pack("<I", (rsrc1 & ~0x3F) | cand) + kd[52:]
                if data.find(probe) >= 0:
                    out[name] = (cand + 1) * 8
                    break
    return out


def find_files(d):
    s = [os.path.join(d, f) for f in os.listdir(d) if f.endswith(".s") and "amdgcn" in f]
    o = [os.path.join(d, f) for f in os.listdir(d) if f.endswith(".out") and "amdgcn" in f]
    return sorted(s), sorted(o)


def audit(d, kernel_filter=None, show_hazards=False, quiet=False):
    """Rows per kernel; returns (rows, hazards)."""
    rows, all_h = [], []
    s_files, o_files = find_files(d)
    desc = {}
    for o in o_files:
        desc.update(descriptors(o))
    for sf in s_files:
        asm = open(sf).read()
        fields = kernel_fields(asm)
        wgs = max_workgroup_sizes(asm)
        for name, lines in split_units(asm).items():
            if kernel_filter and kernel_filter not in name:
                continue
            insns, labels = parse(lines)
            top, ldst = top_reg_info(insns)
            hz = analyse(insns, labels, name)
            f = fields.get(name, {})
            dd = desc.get(name)
            raw = [h for h in hz if h[5] == "raw"]
            first = insns[0].text if insns else ""
            rows.append(dict(name=name, kernel=name in fields, next_free_vgpr=f.get("next_free_vgpr"),
                             accum_offset=f.get("accum_offset"), top=top, top_is_load_dst=top in ldst,
                             alloc=dd[1] if dd else None, wg_size=wgs.get(name), kd_accum=dd[2] if dd else None, hazards=len(raw),
                             waw=len(hz) - len(raw),
                             entry_wait=name in fields or first.startswith("s_waitcnt vmcnt(0) expcnt(0) lgkmcnt(0)")))
            all_h += hz
    if not quiet:
        for r in rows:
            print(f"{r['name'][:90]:90s} kernel={int(r['kernel'])} nfv={r['next_free_vgpr']} acc={r['accum_offset']} "
                  f"top=v{r['top']} load_dst={int(r['top_is_load_dst'])} alloc={r['alloc']} hazards={r['hazards']} "
                  f"waw={r['waw']} entry_wait={int(r['entry_wait'])}")
        if show_hazards:
            for h in all_h:
                print("HAZARD" if h[5] == "raw" else "waw", h[0][:60], "insn", h[1], h[2], "regs", h[3][:8],
                      "pending from insn", h[4])
    return rows, all_h


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel")
    ap.add_argument("--hazards", action="store_true")
    a = ap.parse_args(argv)
    rows, hz = audit(a.dir, a.kernel, a.hazards)
    return 1 if any(h[5] == "raw" for h in hz) or not all(r["entry_wait"] for r in rows) else 0


if __name__ == "__main__":
    sys.exit(main())
