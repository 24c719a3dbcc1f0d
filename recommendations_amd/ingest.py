"""Id ingest: drop-in for commons/feature_utils.py:21-46, 136-183.

Same function names, arguments and results as the reference, with the per-id
work (xxHash32 seeds, xxHash64 ids, the history hash / drop-label / cap / pad
loop) in native code (csrc/ingest.hip, C ABI in include/lthm.h) instead of
pandas ``.apply`` loops:

    hash_feature_name_to_int("product_id") == 396283771
    hash_string_to_long("12345", 396283771, False) == -7448648811083631205

Values are converted with Python ``str()`` exactly as the reference does;
int64 arrays skip that step (their decimal form is produced natively, also on
the GPU via :func:`hash_int64_ids_device`).
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np

from ._lib import call, load

MAX_LONG_VALUE_PLUS_ONE = 2 ** 63
CATEGORICAL_VAR_HASH_PAD_TOKEN = 0


def _lib():
    return load()


def to_lower_case(name: str) -> str:
    return name.lower()


def hash_feature_name_to_int(feature_name: str) -> int:
    """feature_utils.py:36-37: xxh32(lower(name), seed 0)."""
    b = to_lower_case(feature_name).encode("utf-8")
    return int(_lib().lthm_xxh32(b, len(b), 0))


def hash_string_to_long(arg, seed: int, value_to_lower: bool) -> int:
    """feature_utils.py:40-46: xxh64(str(arg), seed) - 2^63."""
    s = str(arg)
    if value_to_lower:
        s = s.lower()
    b = s.encode("utf-8")
    return int(_lib().lthm_xxh64(b, len(b), int(seed) & 0xFFFFFFFFFFFFFFFF)) - MAX_LONG_VALUE_PLUS_ONE


def _pack(strings: Sequence[str]):
    enc = [s.encode("utf-8") for s in strings]
    lens = np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc))
    offsets = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
    return buf, offsets


def hash_values(values: Iterable, seed: int, value_to_lower: bool) -> np.ndarray:
    """Vectorised hash_string_to_long over a column of values -> int64 [n]."""
    if isinstance(values, np.ndarray) and values.dtype.kind in "iu" and values.dtype.itemsize <= 8:
        vals = np.ascontiguousarray(values, dtype=np.int64)
        if values.dtype == np.uint64:
            raise TypeError("uint64 values: str() differs from int64; pass them as Python ints")
        out = np.empty(vals.shape[0], dtype=np.int64)
        rc = _lib().lthm_hash_int64_str(vals.ctypes.data, vals.shape[0], int(seed) & 0xFFFFFFFFFFFFFFFF,
                                        out.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"lthm_hash_int64_str failed ({rc})")
        return out
    strings = [str(v) for v in values]
    n = len(strings)
    out = np.empty(n, dtype=np.int64)
    if n == 0:
        return out
    buf, offsets = _pack(strings)
    flags = np.zeros(n, dtype=np.uint8)
    nflag = _lib().lthm_hash_strings(buf.ctypes.data, offsets.ctypes.data, n, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                     int(bool(value_to_lower)), out.ctypes.data, flags.ctypes.data)
    if nflag < 0:
        raise RuntimeError("lthm_hash_strings failed")
    if nflag:  # non-ASCII strings: Unicode lowering as Python's str.lower()
        for i in np.nonzero(flags)[0]:
            out[i] = hash_string_to_long(strings[i], seed, True)
    return out


def pad_array(arr, size: int, pad_token: int = CATEGORICAL_VAR_HASH_PAD_TOKEN) -> np.ndarray:
    """feature_utils.py:21-25: int64, truncated to size, right-padded."""
    a = np.array(arr, dtype=np.int64).reshape(-1)
    out = np.empty(size, dtype=np.int64)
    offs = np.array([0, a.shape[0]], dtype=np.int64)
    rc = _lib().lthm_history_pad(a.ctypes.data, offs.ctypes.data, 1, None, 0, size, int(pad_token), out.ctypes.data)
    if rc != 0:
        raise RuntimeError("lthm_history_pad failed")
    return out


def pad_histories(histories: Sequence, length: int, history_id: Optional[np.ndarray] = None,
                  pad_token: int = CATEGORICAL_VAR_HASH_PAD_TOKEN) -> np.ndarray:
    """Rows of already-hashed int64 ids -> [n_rows, length] (drop == history_id[r] when given)."""
    rows = [np.asarray(h, dtype=np.int64).reshape(-1) for h in histories]
    offs = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum([r.shape[0] for r in rows], out=offs[1:])
    items = np.concatenate(rows) if rows and offs[-1] > 0 else np.zeros(1, dtype=np.int64)
    out = np.empty((len(rows), length), dtype=np.int64)
    hid = None if history_id is None else np.ascontiguousarray(history_id, dtype=np.int64)
    rc = _lib().lthm_history_pad(items.ctypes.data, offs.ctypes.data, len(rows),
                                 hid.ctypes.data if hid is not None else None, int(hid is not None), length,
                                 int(pad_token), out.ctypes.data)
    if rc != 0:
        raise RuntimeError("lthm_history_pad failed")
    return out


def xxhash_categorical_values_to_number(batch, column: str, value_to_lower: bool):
    """feature_utils.py:136-142 (pandas DataFrame in place)."""
    seed = hash_feature_name_to_int(feature_name=column)
    batch[column] = hash_values(batch[column].values, seed, value_to_lower)


def handle_categorical_history_feature(batch, column: str, hash_ids: bool, history_length: int,
                                       history_id_feature_name: str, remove_history_id_from_history: bool = False):
    """feature_utils.py:149-179 (pandas DataFrame in place)."""
    if not hash_ids and not remove_history_id_from_history:
        return truncate_and_pad_to_fix_len(batch=batch, column=column, length=history_length)
    seed = hash_feature_name_to_int(feature_name=history_id_feature_name)
    histories = list(batch[column].values)
    if hash_ids:
        flat = [h for hist in histories for h in hist]
        hashed = hash_values(flat, seed, False) if flat else np.zeros(0, dtype=np.int64)
        rows, k = [], 0
        for hist in histories:
            rows.append(hashed[k:k + len(hist)])
            k += len(hist)
    else:
        rows = histories
    hid = np.asarray(batch[history_id_feature_name].values, dtype=np.int64) if remove_history_id_from_history else None
    out = pad_histories(rows, history_length, hid)
    batch[column] = list(out)


def truncate_and_pad_to_fix_len(batch, column: str, length: int):
    """feature_utils.py:182-183."""
    batch[column] = list(pad_histories(list(batch[column].values), length))


def hash_int64_ids_device(ids, seed: int):
    """hash_string_to_long(str(id), seed) for an int64 CUDA tensor, on the GPU."""
    import torch
    from ._lib import ptr, require_gpu, stream
    require_gpu(ids)
    if ids.dtype != torch.int64:
        raise TypeError("int64 ids expected")
    out = torch.empty_like(ids)
    call("lthm_hash_int64_str_dev", ptr(ids), ids.numel(), int(seed) & 0xFFFFFFFFFFFFFFFF, ptr(out), stream())
    return out
