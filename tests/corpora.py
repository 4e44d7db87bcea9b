"""Synthetic compression corpora shared by the GPU zstd tests, bench.py and
tools/ (test and benchmark data, not product code).  All deterministic.

* text     a 2 000-word vocabulary of random lowercase words, words drawn
           uniformly, space separated (the bench's encode corpus)
* records  CSV-like rows: ids, two names from 300, amounts, dates
* far      long repeats 256 KiB - 1 MiB back over a text / records / binary base
* code     C-source-like text (kernel_tree: the configs[3] file mix built on it)
* binary   a mix of the byte shapes a backup holds besides text: fixed-width
           little-endian structs (incrementing ids, small counters, float32
           measurements with shared exponents, zero-padded name fields, flag
           bytes), runs of code-like bytes (opcode templates with random
           immediates and displacements) and short incompressible stretches
           (compressed or encrypted payloads), interleaved in 1-16 KiB pieces;
           bytes >= 128 throughout (it is the corpus that exercises
           Huffman literals with FSE-compressed weights)
"""
import numpy as np


def text(n: int, seed: int = 21) -> np.ndarray:
    rng = np.random.default_rng(seed)
    vocab = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 11, 2000)]
    t = b" ".join(vocab[i] for i in rng.integers(0, 2000, n // 4 + 16))
    return np.frombuffer(t[:n], np.uint8).copy()


def records(n: int, seed: int = 3) -> np.ndarray:
    """CSV-like rows (ids, names, amounts, dates): long repeats at varied
    offsets and skewed codes."""
    rng = np.random.default_rng(seed)
    names = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(4, 12, 300)]
    m = n // 24 + 16  # rows (>= 25 bytes each)
    a, b = rng.integers(0, 300, m), rng.integers(0, 300, m)
    x, y, d = rng.integers(0, 1000, m), rng.integers(0, 100, m), rng.integers(1, 29, m)
    t = b"".join(b"%d,%s,%s,%d.%02d,2026-10-%02d\n" % (100000 + i, names[a[i]], names[b[i]], x[i], y[i], d[i])
                 for i in range(m))
    return np.frombuffer(t[:n], np.uint8).copy()


def _structs(rng, nbytes: int, id0: int) -> bytes:
    m = nbytes // 48 + 1
    rec = np.zeros(m, dtype=[("id", "<u4"), ("count", "<u2"), ("kind", "u1"), ("flags", "u1"),
                             ("value", "<f4"), ("scale", "<f4"), ("stamp", "<u8"), ("name", "S16"),
                             ("pad", "<u4"), ("crc", "<u4")])
    rec["id"] = np.arange(id0, id0 + m, dtype=np.uint32)
    rec["count"] = rng.integers(0, 40, m)
    rec["kind"] = rng.choice(np.array([1, 2, 3, 7, 0x81, 0xC0], np.uint8), m)
    rec["flags"] = rng.choice(np.array([0, 0, 0x80, 0x01, 0xFF], np.uint8), m)
    rec["value"] = (rng.normal(100.0, 3.0, m)).astype(np.float32)
    rec["scale"] = rng.choice(np.array([0.5, 1.0, 2.0, 1000.0], np.float32), m)
    rec["stamp"] = 1_790_000_000_000 + np.cumsum(rng.integers(1, 5000, m)).astype(np.uint64)
    names = [b"alpha", b"beta", b"gamma_ray", b"delta.cfg", b"\xc3\xa9t\xc3\xa9", b"omega-7", b"", b"sigma.log"]
    rec["name"] = [names[i] for i in rng.integers(0, len(names), m)]
    rec["crc"] = rng.integers(0, 1 << 32, m, dtype=np.uint64).astype(np.uint32)
    return rec.tobytes()[:nbytes]


_OPS = [b"\x48\x89\xe5", b"\x48\x83\xec", b"\x48\x8b\x45", b"\x48\x8d\x05", b"\xe8", b"\xe9", b"\x0f\x84",
        b"\x0f\x85", b"\x41\x57", b"\x41\x56", b"\x55", b"\x5d", b"\xc3", b"\x31\xc0", b"\x48\x85\xc0",
        b"\x74", b"\x75", b"\x89\x45", b"\x8b\x45", b"\xff\x15", b"\x66\x0f\x1f\x44\x00\x00", b"\x90"]
_IMM = [0, 0, 1, 2, 4, 8, 1, 2, 4, 4]  # immediate bytes after each template (cycled)


def _code(rng, nbytes: int) -> bytes:
    out = bytearray()
    ops = rng.integers(0, len(_OPS), nbytes // 3 + 8)
    for k, o in enumerate(ops):
        out += _OPS[o]
        w = _IMM[(o + k) % len(_IMM)] if o in (1, 2, 3, 4, 5, 6, 7, 15, 16, 17, 18, 19) else 0
        if w:
            v = int(rng.integers(-200, 200)) if w <= 2 else int(rng.integers(-(1 << 20), 1 << 20))
            out += (v & ((1 << (8 * w)) - 1)).to_bytes(w, "little")
        if len(out) >= nbytes:
            break
    return bytes(out[:nbytes])


def binary(n: int, seed: int = 5) -> np.ndarray:
    rng = np.random.default_rng(seed)
    parts, at, id0 = [], 0, 1000
    while at < n:
        k = int(rng.integers(1 << 10, 16 << 10))
        r = rng.random()
        if r < 0.5:
            b = _structs(rng, k, id0)
            id0 += k // 48 + 1
        elif r < 0.85:
            b = _code(rng, k)
        else:
            b = rng.integers(0, 256, min(k, 4096), dtype=np.uint8).tobytes()
        parts.append(b)
        at += len(b)
    return np.frombuffer(b"".join(parts)[:n], np.uint8).copy()


def far(n: int, seed: int = 31) -> np.ndarray:
    """Long repeats at 256 KiB - 1 MiB distances (the 2^20 window of
    SecureStorage::compress, storage.rs:74-84, at mapache's 512K/1M/8M
    chunks): a base of 32 KiB pieces taken in turn from text, records and
    binary, then, every 4-64 KiB, a 1-32 KiB stretch overwritten by a copy of
    the bytes 256 KiB - 1 MiB before it (about a third of the bytes), as in a
    tree of near-duplicate files."""
    rng = np.random.default_rng(seed)
    src = [text(n, seed + 1), records(n, seed + 2), binary(n, seed + 3)]
    out = np.empty(n, np.uint8)
    for k, o in enumerate(range(0, n, 32768)):
        out[o:o + 32768] = src[k % 3][o:o + 32768]
    pos = 256 << 10
    while pos < n:
        pos += int(rng.integers(4 << 10, 64 << 10))
        ln, d = int(rng.integers(1 << 10, 32 << 10)), int(rng.integers(256 << 10, 1 << 20))
        if pos - d < 0 or pos + ln > n:
            continue
        out[pos:pos + ln] = out[pos - d:pos - d + ln]
        pos += ln
    return out


_KW = [b"static", b"int", b"unsigned", b"long", b"void", b"struct", b"const", b"return", b"if", b"else", b"for",
       b"while", b"goto", b"break", b"case", b"switch", b"sizeof", b"u32", b"u64", b"bool", b"NULL", b"err", b"ret"]


def code(n: int, seed: int = 41) -> np.ndarray:
    """C-source-like text: functions of indented statements over a Zipf-skewed
    identifier vocabulary (kernel-tree-like bytes for configs[3])."""
    rng = np.random.default_rng(seed)
    idents = [b"_".join(bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 7, int(w)))
              for w in rng.integers(1, 4, 5000)]
    m = n // 24 + 64  # lines drawn (>= 25 bytes each on average)
    z = np.minimum(rng.zipf(1.3, (m, 4)) - 1, len(idents) - 1)
    kw, hdr, close = rng.integers(0, len(_KW), (m, 2)), rng.random(m) < 0.08, rng.random(m) < 0.1
    depth, nk, op = rng.integers(1, 4, m), rng.integers(1, 4, m), rng.integers(0, 9, (m, 3))
    ops = [b" = ", b" + ", b" & ", b" == ", b" != ", b"->", b", ", b" | ", b" < "]
    tabs = [b"\t" * d for d in range(4)]
    out, at, i = [], 0, 0
    while at < n:
        zi, ki = z[i % m], kw[i % m]
        if hdr[i % m]:  # a function header
            line = b"\n%s %s(struct %s *%s, %s %s)\n{\n" % (_KW[ki[0] % 6], idents[zi[0]], idents[zi[1]],
                                                           idents[zi[2]], _KW[ki[1] % 6], idents[zi[3]])
        else:
            d, k, oi = int(depth[i % m]), int(nk[i % m]), op[i % m]
            expr = idents[zi[0]] + b"".join(ops[oi[t]] + idents[zi[t + 1]] for t in range(k))
            line = tabs[d] + (_KW[ki[0]] + b" (" + expr + b")\n" if ki[0] < 11 else expr + b";\n")
            if close[i % m]:
                line += tabs[d - 1] + b"}\n"
        out.append(line)
        at += len(line)
        i += 1
    return np.frombuffer(b"".join(out)[:n], np.uint8).copy()


def kernel_tree(nfiles: int = 80000, seed: int = 2025):
    """BASELINE configs[3] stand-in ("extracted Linux kernel source tree, ~80 k
    small files, dedup-heavy realistic mix"; no tree here or on the GPU box):
    file sizes log-normal (median 8 KiB, sigma 1.2, at most 64 MiB: ~1.3 GB for
    80 000 files), each file a license line, its own name line, then C-like
    text (`code`) taken from a 16 MiB base at a random offset; about 10 % of
    the files are exact copies of an earlier file (dedup at blob level).
    Returns (arena, offsets, lengths, duplicate_of: -1 or the copied file)."""
    rng = np.random.default_rng(seed)
    sizes = np.minimum(np.exp(rng.normal(np.log(8192), 1.2, nfiles)).astype(np.int64) + 1, 64 << 20)
    dup = np.where(rng.random(nfiles) < 0.1, (rng.random(nfiles) * np.arange(nfiles)).astype(np.int64), -1)
    dup[0] = -1
    for f in np.nonzero(dup >= 0)[0]:  # (in file order: a copy of a copy has its final size)
        sizes[f] = sizes[dup[f]]
    base = code(16 << 20, seed)
    bb = np.concatenate([base, base])
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    out = np.empty(int(sizes.sum()), np.uint8)
    starts = rng.integers(0, base.size, nfiles)
    for f in range(nfiles):
        o, ln = int(offs[f]), int(sizes[f])
        if dup[f] >= 0:
            d = int(dup[f])
            out[o:o + ln] = out[int(offs[d]):int(offs[d]) + ln]
            continue
        hdr = (b"// SPDX-License-Identifier: GPL-2.0\n/* drivers/%d/%d.c */\n" % (f % 977, f))[:ln]
        h = len(hdr)
        out[o:o + h] = np.frombuffer(hdr, np.uint8)
        rest = ln - h
        while rest > 0:  # (files above 32 MiB wrap the base)
            s0 = int(starts[f]) % base.size
            k = min(rest, base.size)
            out[o + ln - rest:o + ln - rest + k] = bb[s0:s0 + k]
            rest -= k
    return out, offs.astype(np.uint64), sizes.astype(np.uint64), dup


def by_name(kind: str, n: int, seed: int | None = None) -> np.ndarray:
    f = {"text": text, "records": records, "binary": binary, "far": far, "code": code}[kind]
    return f(n) if seed is None else f(n, seed)
