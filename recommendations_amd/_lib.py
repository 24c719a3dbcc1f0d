"""ctypes binding of the C ABI declared in ``include/lthm.h``.

The prototypes are parsed from the header itself, so the Python side can never
drift from the ABI a cgo/JNI/ctypes integrator would bind.
There is deliberately no CPU fallback: every product op calls into
``liblthm_hip.so`` and raises if the library or a GPU is missing.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Dict, List, Tuple

import torch  # noqa: F401  (loads torch's libamdhip64 first, so the .so binds to the same HIP runtime)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(_PKG_DIR)
HEADER = os.path.join(REPO_ROOT, "include", "lthm.h")
# LTHM_LIB_PATH: another in-tree build of the same library, for A/B measurements of a kernel change
LIB_PATH = os.environ.get("LTHM_LIB_PATH") or os.path.join(_PKG_DIR, "liblthm_hip.so")

F32 = 0
BF16 = 1
DTYPE_CODE = {torch.float32: F32, torch.bfloat16: BF16}

_CTYPE = {
    "int64_t*": ctypes.c_void_p,
    "int32_t*": ctypes.c_void_p,
    "uint8_t*": ctypes.c_void_p,
    "uint16_t*": ctypes.c_void_p,
    "uint64_t*": ctypes.c_void_p,
    "float*": ctypes.c_void_p,
    "void*": ctypes.c_void_p,
    "char*": ctypes.c_char_p,
    "char**": ctypes.c_void_p,
    "float**": ctypes.c_void_p,
    "void**": ctypes.c_void_p,
    "int64_t": ctypes.c_int64,
    "uint64_t": ctypes.c_uint64,
    "int32_t": ctypes.c_int32,
    "uint32_t": ctypes.c_uint32,
    "int": ctypes.c_int,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "size_t": ctypes.c_size_t,
}


def parse_header(path: str = HEADER) -> Dict[str, Tuple[str, List[str]]]:
    """Return {name: (return type, [arg types])} for every prototype in lthm.h."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    text = re.sub(r"#[^\n]*", " ", text)
    protos = {}
    for m in re.finditer(r"\b(int|void|int64_t|uint32_t|uint64_t|double|float)\s+(lthm_\w+)\s*\(([^)]*)\)\s*;",
                         text, flags=re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        types = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.replace("const ", "").split())
                # drop the parameter name, keep pointer stars
                tm = re.match(r"^([A-Za-z_0-9]+)\s*(\**)\s*[A-Za-z_0-9]*$", a.replace(" *", "*").replace("* ", "* "))
                if tm is None:
                    base = a.split()[0]
                    stars = a.count("*")
                else:
                    base, stars = tm.group(1), len(tm.group(2))
                    stars = a.count("*")
                types.append(base + "*" * stars)
        protos[name] = (ret, types)
    return protos


def parse_structs(path: str = HEADER) -> Dict[str, type]:
    """ctypes.Structure classes for every `typedef struct name {...} name;` in lthm.h."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    out = {}
    for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*(\w+)\s*;", text, flags=re.S):
        fields = []
        for line in m.group(2).split(";"):
            line = " ".join(line.replace("const ", "").split())
            if not line:
                continue
            typ, name = line.rsplit(" ", 1)
            stars = name.count("*") + typ.count("*")
            typ, name = typ.replace("*", "").strip(), name.replace("*", "")
            ct = _CTYPE[typ + "*" * stars]
            am = re.match(r"^(\w+)\[(\d+)\]$", name)
            if am:
                name, ct = am.group(1), ct * int(am.group(2))
            fields.append((name, ct))
        out[m.group(3)] = type(m.group(3), (ctypes.Structure,), {"_fields_": fields})
    return out


STRUCTS = parse_structs()
for _n in STRUCTS:
    _CTYPE[_n + "*"] = ctypes.c_void_p

_LIB = None
_PROTOS: Dict[str, Tuple[str, List[str]]] = {}


def load() -> ctypes.CDLL:
    global _LIB, _PROTOS
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: the HIP extension is not built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'`). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    protos = parse_header()
    for name, (ret, args) in protos.items():
        fn = getattr(lib, name)
        fn.restype = {"int": ctypes.c_int, "void": None, "int64_t": ctypes.c_int64, "uint32_t": ctypes.c_uint32,
                      "uint64_t": ctypes.c_uint64, "double": ctypes.c_double, "float": ctypes.c_float}[ret]
        fn.argtypes = [_CTYPE[a] for a in args]
    _LIB, _PROTOS = lib, protos
    return lib


TORCH_OPS_PATH = os.path.join(_PKG_DIR, "liblthm_torch_ops.so")
_TORCH_OPS = False


def load_torch_ops() -> None:
    """Register the TORCH_LIBRARY(lthm) ops (csrc/torch_ops/lthm_ops.cpp) with the
    dispatcher: the scriptable boundary (torch.ops.lthm.*) over the same kernels.
    Raises if the op library is not built (no fallback)."""
    global _TORCH_OPS
    if _TORCH_OPS:
        return
    if not os.path.exists(TORCH_OPS_PATH):
        raise RuntimeError(
            f"{TORCH_OPS_PATH} not found: the TORCH_LIBRARY(lthm) op layer is not built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'`).")
    lib = load()  # liblthm_hip.so first (RTLD_GLOBAL), the op library links against it
    torch.ops.load_library(TORCH_OPS_PATH)
    # the op library fills the descriptors of include/lthm.h: a stale build (older header)
    # would hand the kernels a shorter struct, so refuse it
    built, want = int(torch.ops.lthm.built_abi_version()), int(lib.lthm_abi_version())
    if built != want:
        raise RuntimeError(f"{TORCH_OPS_PATH} was built against ABI {built}, liblthm_hip.so is ABI {want}: "
                           "rebuild it (`python recommendations_amd/csrc/torch_ops/build.py`)")
    _TORCH_OPS = True


class KernelTimer:
    """Live per-entry-point timing with HIP events on torch's current stream (the
    stream every launch goes to).  bench.py enables it over the timed region;
    ``work`` is the algorithmic bytes / flops the wrapper declares per call, or a
    callable evaluated in summary() for data-dependent work (e.g. touched rows)."""

    def __init__(self, only=None):
        self.records = []  # (key, ev0, ev1, work, unit, bytes)
        self.only = None if only is None else set(only)  # time just these keys (others run untouched)

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for key, e0, e1, work, unit, nbytes in self.records:
            s = out.setdefault(key, {"calls": 0, "ms": 0.0, "work": 0.0, "unit": unit, "bytes": 0.0})
            s["calls"] += 1
            s["ms"] += e0.elapsed_time(e1)
            if callable(work):  # data-dependent work (a device count snapshot), read after the timed region
                work = work()
            s["work"] += work or 0.0
            s["bytes"] += nbytes or 0.0
        return out


TIMER = None  # type: KernelTimer


def call(name: str, *args, _key: str = None, _work: float = None, _unit: str = None, _bytes: float = None) -> None:
    lib = load()
    t = TIMER
    if t is not None and (t.only is None or (_key or name) in t.only):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(lib, name)(*args)
        e1.record()
        t.records.append((_key or name, e0, e1, _work, _unit, _bytes))
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with hip error {rc}")


def sub_events(key: str, work: float = None, unit: str = None, nbytes: float = None):
    """(start, end) HIP events for ONE kernel launched inside a C-ABI call, which records them
    around that launch (e.g. lthm_contrastive_desc.main_ev0 / main_ev1), or None when the live
    timer is off or does not want ``key``.  Both events are recorded here once first, so their
    handles exist; the call re-records them at the kernel's boundaries."""
    t = TIMER
    if t is None or (t.only is not None and key not in t.only):
        return None
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()
    t.records.append((key, e0, e1, work, unit, nbytes))
    return e0, e1


def timer_on() -> bool:
    return TIMER is not None


def TIMER_RECORDS() -> list:
    """The live timer's records (key, ev0, ev1, work, unit, bytes) as mutable lists, or [] when the
    timer is off: a wrapper replaces a record's work by a callable once the device knows it."""
    t = TIMER
    if t is None:
        return []
    for i, r in enumerate(t.records):
        if not isinstance(r, list):
            t.records[i] = list(r)
    return t.records


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int:
    if t is None:
        return None
    return t.data_ptr()


def dcode(t: torch.Tensor) -> int:
    try:
        return DTYPE_CODE[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}; the gfx950 kernels take float32 or bfloat16")


def require_gpu(*tensors) -> None:
    """Fail loudly: the product path has no CPU fallback."""
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "recommendations_amd ops run only on an MI355X (gfx950) device; got a CPU tensor. "
                "The CPU restatement lives in oracle/ and is test infrastructure only.")
        if not t.is_contiguous():
            raise RuntimeError("recommendations_amd ops require contiguous tensors")
