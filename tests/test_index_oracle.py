"""CPU: the dedup-index restatement (oracle.DedupIndex) against hand-written
cases of Repository::save_blob's check (repository_v1.rs:169-180)."""
import numpy as np

from oracle import oracle as O


def _id(b: int, tail: int = 0) -> np.ndarray:
    a = np.zeros(32, np.uint8)
    a[0], a[31] = b, tail
    return a


def test_first_occurrence_in_order_within_and_across_batches():
    ix = O.DedupIndex()
    b1 = np.stack([_id(1), _id(2), _id(1), _id(3), _id(2)])
    assert ix.add(b1).tolist() == [True, True, False, True, False]
    b2 = np.stack([_id(3), _id(4), _id(4), _id(1, 9)])  # (1, 9): same prefix as (1, 0), another ID
    assert ix.add(b2).tolist() == [False, True, False, True]
    assert len(ix) == 5
    assert ix.add(np.zeros((0, 32), np.uint8)).tolist() == []


def test_pack_plan_and_header_restatement():
    """repository_v1.rs:185-193 (flush after the add that passes the limit, then
    the rest) and packer.rs:156-186 (37-byte entries, padding to 64)."""
    assert O.pack_plan([5, 5, 5, 5, 5], 9) == [(0, 2), (2, 4), (4, 5)]
    assert O.pack_plan([10], 9) == [(0, 1)] and O.pack_plan([9, 1], 9) == [(0, 2)] and O.pack_plan([], 9) == []
    ids = np.arange(64, dtype=np.uint8).reshape(2, 32)
    h = O.pack_header(ids, [300, 70000], [0, 1], [bytes(range(36))])
    assert len(h) == 3 * 37 and h[32:37] == (300).to_bytes(4, "little") + b"\x00"
    assert h[37 + 32:37 + 37] == (70000).to_bytes(4, "little") + b"\x01" and h[-1] == 0xFF
