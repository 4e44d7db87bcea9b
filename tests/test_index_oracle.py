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
