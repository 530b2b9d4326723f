"""Python binding for the hand-written CDNA4 (gfx950) HIP kernel library.

The kernels live in ``ops/csrc/*.hip`` and are compiled with ``hipcc --offload-arch=gfx950``
into ONE in-tree shared library, ``ops/_lib/libdlms_hip.so`` (plain C ABI, no torch headers,
seconds to build).  It is loaded with ``ctypes`` AFTER ``torch`` so that it binds to the HIP
runtime torch already loaded (same SONAME ``libamdhip64.so.7``), hence shares streams, the
caching allocator's memory and hipGraph capture with torch.

Every wrapper checks shapes/dtypes/devices on the host before launching (a bad launch on the
box can reset the GPU), launches on ``torch.cuda.current_stream()`` and raises on any HIP
error.  There is deliberately NO silent PyTorch fallback: if the library is missing on a GPU
host, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from pathlib import Path

import torch

_HERE = Path(__file__).resolve().parent
CSRC = _HERE / "csrc"
LIB_DIR = _HERE / "_lib"
LIB_PATH = LIB_DIR / "libdlms_hip.so"
# debug variant: device-side range checks on every data-dependent index (common.h, DLMS_DEVICE_CHECKS)
CHECKED_LIB_PATH = LIB_DIR / "libdlms_hip_checked.so"
CHECK_UNITS = ("gemm", "attention", "decode", "encoder", "skinny", "gemm_ps")
CHECK_SITES = {1: "embed token id", 2: "position id", 3: "decode_update slot_map", 4: "decode_update token id",
               5: "decode_update sequence length", 6: "seen_set row", 7: "QKV scatter slot", 8: "QKV scatter position",
               9: "attention slot", 10: "BERT token id", 11: "seen_set token id"}
SOURCES = ["api.hip", "gemm.hip", "norm.hip", "attention.hip", "decode.hip", "encoder.hip", "xgmi.hip", "skinny.hip", "gemm_ps.hip",
           "dataflow.hip", "mid.hip"]
ARCH = os.environ.get("DLMS_OFFLOAD_ARCH", "gfx950")

EPI_BF16, EPI_GELU_TANH, EPI_GELU_ERF, EPI_F32, EPI_QKV, EPI_ARGMAX, EPI_PARTIAL = range(7)

_lock = threading.Lock()
_lib = None


def _sources() -> list[Path]:
    return [CSRC / s for s in SOURCES]


def checked_mode() -> bool:
    """``DLMS_KERNEL_CHECKS=1`` loads the range-checked debug build instead of the production one."""
    return os.environ.get("DLMS_KERNEL_CHECKS", "0") not in ("", "0")


def needs_build(checked: bool = False) -> bool:
    path = CHECKED_LIB_PATH if checked else LIB_PATH
    if not path.exists():
        return True
    t = path.stat().st_mtime
    deps = _sources() + list(CSRC.glob("*.h"))
    return any(p.stat().st_mtime > t for p in deps)


def build(force: bool = False, verbose: bool = False, checked: bool = False, out: str | None = None,
          defines: tuple[str, ...] = ()) -> Path:
    """Compile every kernel source for gfx950 into the in-tree shared library (``checked``: the
    debug variant with device-side index range checks, ``-DDLMS_DEVICE_CHECKS=1``).  ``out`` +
    ``defines`` (``NAME=VALUE``): an A/B variant for experiments (loaded via ``DLMS_HIP_LIB``)."""
    path = Path(out) if out else (CHECKED_LIB_PATH if checked else LIB_PATH)
    if not out and not force and not needs_build(checked):
        return path
    path.parent.mkdir(parents=True, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = path.with_suffix(f".so.tmp{os.getpid()}")
    flags = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wno-unused-result"] + \
        (["-DDLMS_DEVICE_CHECKS=1"] if checked else []) + [f"-D{d}" for d in defines]
    # one hipcc per translation unit, in parallel (the kernels of a unit never call another
    # unit's device code, so no relocatable device code is needed), then one link
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    jobs = max(1, min(len(_sources()), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with tempfile.TemporaryDirectory(prefix="dlms_build_") as td:
        objs = [os.path.join(td, src.stem + ".o") for src in _sources()]

        def compile_one(i):
            cmd = [hipcc] + flags + ["-c", str(_sources()[i]), "-o", objs[i]]
            if verbose:
                print(" ".join(cmd), flush=True)
            return subprocess.run(cmd, capture_output=True, text=True)

        with ThreadPoolExecutor(jobs) as ex:
            for src, res in zip(_sources(), ex.map(compile_one, range(len(objs)))):
                if res.returncode != 0:
                    raise RuntimeError(f"hipcc failed on {src.name} ({res.returncode}):\n{res.stderr[-4000:]}")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", str(tmp)] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc link failed ({res.returncode}):\n{res.stderr[-4000:]}")
    os.replace(tmp, path)
    return path


FP8 = torch.float8_e4m3fn  # OCP e4m3 (gfx950), not the MI300 fnuz variant


class GemmEpi(ctypes.Structure):
    _fields_ = [
        ("bias", ctypes.c_void_p), ("out", ctypes.c_void_p), ("ldo", ctypes.c_int),
        ("resid", ctypes.c_void_p), ("ldr", ctypes.c_int),
        ("q_out", ctypes.c_void_p), ("ldq", ctypes.c_int),
        ("k_cache", ctypes.c_void_p), ("v_cache", ctypes.c_void_p),
        ("row_slot", ctypes.c_void_p), ("row_pos", ctypes.c_void_p),
        ("n_heads", ctypes.c_int), ("t_max", ctypes.c_int), ("d_local", ctypes.c_int),
        ("argmax_out", ctypes.c_void_p), ("seen", ctypes.c_void_p),
        ("seen_words", ctypes.c_int), ("vocab", ctypes.c_int), ("col_offset", ctypes.c_int),
        ("penalty", ctypes.c_float),
        ("split_k", ctypes.c_int), ("split_stride", ctypes.c_longlong),
        ("a_scale", ctypes.c_void_p), ("w_scale", ctypes.c_void_p),
        ("n_slots", ctypes.c_int),
    ]


XGMI_MAX_RANKS = 8


class XgmiArgs(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p * XGMI_MAX_RANKS), ("inp", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("n", ctypes.c_longlong), ("slab_bytes", ctypes.c_longlong), ("rank", ctypes.c_int),
                ("world", ctypes.c_int)]


def _bind(L):
    P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    sig = {
        "dlms_gemm": [I, P, I, P, I, I, I, I, ctypes.POINTER(GemmEpi), P],
        "dlms_gemm_fp8": [I, P, I, P, I, I, I, I, ctypes.POINTER(GemmEpi), P],
        "dlms_layernorm": [P, I, P, P, P, I, P, I, I, I, F, P],
        "dlms_layernorm_gather": [P, I, P, P, P, P, I, I, I, F, P],
        "dlms_add_layernorm": [P, I, P, I, ctypes.c_longlong, I, P, P, P, P, I, P, I, P, I, I, F, I, P],
        "dlms_quantize_rows_fp8": [P, I, P, I, P, I, I, P],
        "dlms_row_attention": [P, I, P, P, P, P, P, I, I, I, I, I, F, P],
        "dlms_attention": [P, I, P, P, P, P, P, I, I, I, I, I, F, P],
        "dlms_tile_attention": [P, I, P, P, P, P, P, I, P, I, I, I, I, F, P],
        "dlms_embed": [P, P, P, P, P, I, I, I, I, I, P],
        "dlms_decode_update": [P, I, ctypes.c_longlong, ctypes.c_longlong, P, P, P, P, I, P, I, P, P, P, P, P, P, I, I,
                               I, I, I, I, I, P, P, F, P, I, P],
        "dlms_argmax_reduce": [P, I, ctypes.c_longlong, P, I, P],
        "dlms_seen_set": [P, P, I, P, I, I, P],
        "dlms_bert_embed_ln": [P, P, P, P, P, P, P, P, P, I, I, F, I, I, P],
        "dlms_mean_pool": [P, P, P, P, I, I, P],
        "dlms_cosine": [P, P, P, I, I, I, F, P],
        "dlms_skinny_gemm": [I, P, I, P, P, F, P, I, I, I, ctypes.POINTER(GemmEpi), P],
        "dlms_attention_split": [P, I, P, P, P, P, P, I, I, I, I, I, F, I, I, P, P, I, P],
        "dlms_attention_oproj": [P, I, P, P, P, P, I, I, I, I, F, P, I, I, P, I, ctypes.c_longlong, P],
        "dlms_attention_oproj_grouped": [P, P, P, P, P, I, I, I, I, F, P, I, I, P, ctypes.c_longlong, P],
        "dlms_skinny_addln_gemm": [I, P, P, I, P, I, ctypes.c_longlong, I, P, P, P, F, P, I, I, I,
                                   ctypes.POINTER(GemmEpi), I, ctypes.c_longlong, P, I, P],
        "dlms_skinny_mlp_cg": [I, I, I],
        "dlms_skinny_mlp": [P, I, I, ctypes.c_longlong, P, I, ctypes.c_longlong, I, P, P, P, F, P, P, P, P, P, I,
                            ctypes.c_longlong, I, I, I, I, I, P],
        "dlms_ln_fix": [P, I, ctypes.c_longlong, P, P, F, P, I, I, I, P],
        "dlms_fix_copies": [],
        "dlms_skinny_addln_max_rows": [I],
        "dlms_mid_max_rows": [I],
        "dlms_mid_ln_gemm": [I, P, I, P, P, F, P, I, I, I, ctypes.POINTER(GemmEpi), I, P],
        "dlms_mid_proj": [P, I, P, P, P, I, I, I, I, I, P],
        "dlms_gemm_ps": [I, P, I, P, I, I, I, I, I, I, I, ctypes.POINTER(GemmEpi), P],
        "dlms_attention_persist": [P, I, P, P, P, P, P, I, I, I, I, I, F, I, P],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    # one-shot xGMI collectives (xgmi.hip) and the IPC handle plumbing behind them
    for name, args in {"dlms_xgmi_alloc": [ctypes.c_longlong, I, ctypes.POINTER(ctypes.c_void_p)],
                       "dlms_xgmi_free": [P], "dlms_ipc_get_handle": [P, P],
                       "dlms_ipc_open": [P, ctypes.POINTER(ctypes.c_void_p)], "dlms_ipc_close": [P],
                       "dlms_xgmi_error": [P, I, ctypes.POINTER(ctypes.c_uint)],
                       "dlms_xgmi_error_async": [P, P, P],
                       "dlms_xgmi_allreduce_f32": [ctypes.POINTER(XgmiArgs), P],
                       "dlms_xgmi_allreduce_i64": [ctypes.POINTER(XgmiArgs), P],
                       "dlms_xgmi_allgather_u64": [ctypes.POINTER(XgmiArgs), P]}.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    L.dlms_stream_create_cumask.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.dlms_stream_create_cumask.restype = ctypes.c_int
    L.dlms_stream_destroy.argtypes = [ctypes.c_void_p]
    L.dlms_stream_destroy.restype = ctypes.c_int
    L.dlms_xgmi_header_bytes.restype = ctypes.c_longlong
    for name in ("dlms_ipc_handle_size", "dlms_xgmi_args_size", "dlms_xgmi_max_blocks"):
        getattr(L, name).restype = ctypes.c_int
    for unit in CHECK_UNITS:
        fn = getattr(L, f"dlms_check_{unit}")
        fn.argtypes = [I, ctypes.c_void_p]
        fn.restype = ctypes.c_int
    if L.dlms_xgmi_args_size() != ctypes.sizeof(XgmiArgs):
        raise RuntimeError("XgmiArgs ABI mismatch between ctypes mirror and compiled library")
    L.dlms_gemm_force_tile.argtypes = [ctypes.c_int]
    L.dlms_gemm_force_tile.restype = None
    L.dlms_gemm_tile_count.argtypes = [ctypes.c_int, ctypes.c_int]
    L.dlms_gemm_tile_count.restype = ctypes.c_long
    # in-situ tuning knobs (tests and production leave them unset)
    if os.environ.get("DLMS_GEMM_TILE"):
        L.dlms_gemm_force_tile(int(os.environ["DLMS_GEMM_TILE"]))
    L.dlms_error_string.argtypes = [ctypes.c_int]
    L.dlms_error_string.restype = ctypes.c_char_p
    L.dlms_gemm_epi_size.restype = ctypes.c_int
    if L.dlms_gemm_epi_size() != ctypes.sizeof(GemmEpi):
        raise RuntimeError("GemmEpi ABI mismatch between ctypes mirror and compiled library")


def lib():
    """Load (building first if needed) the kernel library.  Raises if it cannot be loaded."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            checked = checked_mode()
            if needs_build(checked):
                build(checked=checked)
            path = os.environ.get("DLMS_HIP_LIB") or str(CHECKED_LIB_PATH if checked else LIB_PATH)
            L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)  # DLMS_HIP_LIB: A/B builds in experiments
            _bind(L)
            _lib = L
    return _lib


class DlmsCheckRecord(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint), ("site", ctypes.c_int), ("value", ctypes.c_longlong),
                ("bound", ctypes.c_longlong)]


def device_errors(clear: bool = True) -> list[str]:
    """Index violations the checked build recorded since the last call (synchronises the device;
    always empty with the production build, whose kernels carry no checks)."""
    torch.cuda.synchronize()
    out = []
    for unit in CHECK_UNITS:
        rec = DlmsCheckRecord()
        _check(getattr(lib(), f"dlms_check_{unit}")(int(clear), ctypes.byref(rec)), f"dlms_check_{unit}")
        if rec.count:
            out.append(f"{unit}: {rec.count} out-of-range index(es); first: "
                       f"{CHECK_SITES.get(rec.site, rec.site)} = {rec.value} not in [0, {rec.bound})")
    return out


def raise_on_device_errors():
    errs = device_errors()
    if errs:
        raise RuntimeError("kernel index checks failed: " + "; ".join(errs))


def available() -> bool:
    """True when a GPU is present (the HIP library will then be required, not optional)."""
    return torch.cuda.is_available()


def gemm_tile_count(bm: int, bn: int) -> int:
    """Launches of the tiled GEMM issued so far with a ``bm`` x ``bn`` tile (host-side census;
    ``gemm_tile_reset()`` zeroes it): tests assert which instantiation a decode path dispatches."""
    return int(lib().dlms_gemm_tile_count(bm, bn))


def gemm_tile_reset():
    lib().dlms_gemm_tile_count(-1, -1)


def _check(err: int, what: str):
    if err != 0:
        raise RuntimeError(f"{what} failed: HIP error {err} ({lib().dlms_error_string(err).decode()})")


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _req(t: torch.Tensor, dtype, name: str, dim: int | None = None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be on the GPU")
    if dim is not None and t.dim() != dim:
        raise ValueError(f"{name}: expected {dim}-D, got {tuple(t.shape)}")
    if t.dim() >= 1 and t.stride(-1) != 1:
        raise ValueError(f"{name}: last dim must be contiguous")


# ---------------------------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------------------------
def gemm(a: torch.Tensor, w: torch.Tensor, epi: int = EPI_BF16, *, bias=None, out=None, resid=None,
         q_out=None, k_cache=None, v_cache=None, row_slot=None, row_pos=None,
         argmax_out=None, seen=None, vocab: int = 0, col_offset: int = 0, penalty: float = 1.0,
         split_k: int = 1, a_scale=None, w_scale=None):
    """C = a @ w.T with a fused epilogue.  a: bf16 [M, K]; w: bf16 [N, K] (N % 64 == 0, K % 64 == 0).
    fp8 (W8A8): a and w ``torch.float8_e4m3fn`` with f32 ``a_scale`` [M] and ``w_scale`` [N]
    (C = diag(a_scale) (a @ w.T) diag(w_scale)); K % 128 == 0."""
    fp8 = a.dtype == FP8
    _req(a, FP8 if fp8 else torch.bfloat16, "a", 2)
    _req(w, FP8 if fp8 else torch.bfloat16, "w", 2)
    M, K = a.shape
    N, K2 = w.shape
    if K != K2 or K % (128 if fp8 else 64) or N % 64:
        raise ValueError(f"gemm shapes a{tuple(a.shape)} w{tuple(w.shape)}: need matching K%64==0 (fp8: 128), "
                         f"N%64==0")
    ep = GemmEpi()
    if fp8:
        _req(a_scale, torch.float32, "a_scale", 1)
        _req(w_scale, torch.float32, "w_scale", 1)
        if a_scale.numel() < M or w_scale.numel() < N:
            raise ValueError("fp8 scales too short")
        ep.a_scale, ep.w_scale = a_scale.data_ptr(), w_scale.data_ptr()
    if bias is not None:
        _req(bias, torch.float32, "bias", 1)
        if bias.numel() < N:
            raise ValueError("bias too short")
        ep.bias = bias.data_ptr()
    if epi in (EPI_BF16, EPI_GELU_TANH, EPI_GELU_ERF, EPI_F32):
        want = torch.float32 if epi == EPI_F32 else torch.bfloat16
        if out is None:
            out = torch.empty(M, N, dtype=want, device=a.device)
        _req(out, want, "out", 2)
        if out.shape[0] < M or out.shape[1] < N:
            raise ValueError("out too small")
        ep.out, ep.ldo = out.data_ptr(), out.stride(0)
        if resid is not None:
            _req(resid, torch.float32, "resid", 2)
            if resid.shape[0] < M or resid.shape[1] < N:
                raise ValueError("resid too small")
            ep.resid, ep.ldr = resid.data_ptr(), resid.stride(0)
    elif epi == EPI_QKV:
        for t, n in ((q_out, "q_out"), (k_cache, "k_cache"), (v_cache, "v_cache")):
            _req(t, torch.bfloat16, n)
        _req(row_slot, torch.int32, "row_slot", 1)
        _req(row_pos, torch.int32, "row_pos", 1)
        if N % 3:
            raise ValueError("QKV N must be 3*d_local")
        d_local = N // 3
        if d_local % 64:
            raise ValueError("d_local must be a multiple of the 64-wide head")
        if k_cache.dim() != 4 or k_cache.shape != v_cache.shape or k_cache.shape[1] * 64 != d_local or k_cache.shape[3] != 64:
            raise ValueError(f"cache shape {tuple(k_cache.shape)} incompatible with d_local={d_local}")
        if q_out.shape[0] < M or q_out.shape[1] < d_local or row_slot.numel() < M or row_pos.numel() < M:
            raise ValueError("qkv epilogue buffers too small")
        ep.q_out, ep.ldq = q_out.data_ptr(), q_out.stride(0)
        ep.k_cache, ep.v_cache = k_cache.data_ptr(), v_cache.data_ptr()
        ep.row_slot, ep.row_pos = row_slot.data_ptr(), row_pos.data_ptr()
        ep.n_heads, ep.t_max, ep.d_local = k_cache.shape[1], k_cache.shape[2], d_local
        ep.n_slots = k_cache.shape[0]
        out = q_out
    elif epi == EPI_PARTIAL:
        if split_k < 1 or K % ((128 if fp8 else 64) * split_k):
            raise ValueError(f"split_k={split_k} must divide K/64 (K={K})")
        if out is None:
            out = torch.empty(split_k, M, N, dtype=torch.float32, device=a.device)
        _req(out, torch.float32, "out", 3)
        if out.shape[0] < split_k or out.shape[1] < M or out.shape[2] < N:
            raise ValueError("partial out too small")
        ep.out, ep.ldo, ep.split_k, ep.split_stride = out.data_ptr(), out.stride(1), split_k, out.stride(0)
    elif epi == EPI_ARGMAX:
        # argmax_out: int64 [M, >= N/64] partial keys, one per (row, 64-column group of tile starts);
        # columns never written must be zero-initialised once (0 is the minimum key)
        _req(argmax_out, torch.int64, "argmax_out", 2)
        _req(seen, torch.int32, "seen", 2)
        if argmax_out.shape[0] < M or argmax_out.shape[1] < N // 64 or seen.shape[0] < M or \
                seen.shape[1] * 32 < vocab or col_offset % 64:
            raise ValueError("argmax epilogue buffers too small / misaligned shard")
        ep.argmax_out, ep.ldo, ep.seen = argmax_out.data_ptr(), argmax_out.stride(0), seen.data_ptr()
        ep.seen_words, ep.vocab, ep.col_offset, ep.penalty = seen.stride(0), vocab, col_offset, penalty
        out = argmax_out
    else:
        raise ValueError(f"unknown epilogue {epi}")
    # the LDS-staged epilogue stores 16 B per lane: rows and bases must be 16-B aligned
    if epi in (EPI_BF16, EPI_GELU_TANH, EPI_GELU_ERF, EPI_PARTIAL, EPI_QKV):
        t = q_out if epi == EPI_QKV else out
        per = 4 if epi == EPI_PARTIAL else 8
        ld = t.stride(1) if epi == EPI_PARTIAL else t.stride(0)
        if t.data_ptr() % 16 or ld % per or (epi == EPI_PARTIAL and t.stride(0) % per):
            raise ValueError("gemm: output rows must be 16-byte aligned")
        if epi == EPI_QKV and (k_cache.data_ptr() % 16 or v_cache.data_ptr() % 16):
            raise ValueError("gemm: KV cache must be 16-byte aligned")
    if fp8:
        if epi in (EPI_GELU_ERF, EPI_F32):
            raise ValueError("fp8 GEMM: epilogue not instantiated")
        _check(lib().dlms_gemm_fp8(epi, _p(a), a.stride(0), _p(w), w.stride(0), M, N, K, ctypes.byref(ep),
                                   _stream()), "dlms_gemm_fp8")
    else:
        _check(lib().dlms_gemm(epi, _p(a), a.stride(0), _p(w), w.stride(0), M, N, K, ctypes.byref(ep), _stream()),
               "dlms_gemm")
    return out


def quantize_fp8_rows(a: torch.Tensor, out=None, scale=None):
    """bf16 [M, D] -> (e4m3 [M, D], f32 row scales [M]) with scale = absmax / 448 (HIP kernel)."""
    _req(a, torch.bfloat16, "a", 2)
    M, D = a.shape
    if D % 4:
        raise ValueError("quantize_fp8_rows: D % 4")
    out = torch.empty(M, D, dtype=FP8, device=a.device) if out is None else out
    scale = torch.empty(M, dtype=torch.float32, device=a.device) if scale is None else scale
    _req(out, FP8, "out", 2)
    _req(scale, torch.float32, "scale", 1)
    if out.shape[0] < M or out.shape[1] < D or scale.numel() < M or out.stride(0) % 4:
        raise ValueError("quantize_fp8_rows: outputs too small / misaligned")
    _check(lib().dlms_quantize_rows_fp8(_p(a), a.stride(0), _p(out), out.stride(0), _p(scale), M, D, _stream()),
           "dlms_quantize_rows_fp8")
    return out, scale


def quantize_fp8_weight(w: torch.Tensor):
    """Host/torch-side weight quantisation: per-output-channel (row) scale = absmax / 448."""
    wf = w.float()
    scale = (wf.abs().amax(dim=1).clamp_min(1e-20) / 448.0)
    q = (wf / scale[:, None]).clamp(-448.0, 448.0).to(FP8)
    return q.contiguous(), scale.contiguous()

def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, *, out_bf16=None,
              out_f32=None, want_bf16: bool = True):
    _req(x, torch.float32, "x", 2)
    M, D = x.shape
    _req(gamma, torch.float32, "gamma", 1)
    _req(beta, torch.float32, "beta", 1)
    if gamma.numel() != D or beta.numel() != D or D % 4 or D > 2048:
        raise ValueError("layernorm: bad gamma/beta/D")
    if want_bf16 and out_bf16 is None:
        out_bf16 = torch.empty(M, D, dtype=torch.bfloat16, device=x.device)
    if out_bf16 is not None:
        _req(out_bf16, torch.bfloat16, "out_bf16", 2)
        if out_bf16.shape[0] < M or out_bf16.shape[1] < D:
            raise ValueError("out_bf16 too small")
    if out_f32 is not None:
        _req(out_f32, torch.float32, "out_f32", 2)
        if out_f32.shape[0] < M or out_f32.shape[1] < D:
            raise ValueError("out_f32 too small")
    _check(lib().dlms_layernorm(_p(x), x.stride(0), _p(gamma), _p(beta), _p(out_bf16),
                                out_bf16.stride(0) if out_bf16 is not None else 0, _p(out_f32),
                                out_f32.stride(0) if out_f32 is not None else 0, M, D, float(eps), _stream()),
           "dlms_layernorm")
    return out_bf16 if out_bf16 is not None else out_f32


def add_layernorm(x: torch.Tensor, gamma, beta, eps: float, *, parts: torch.Tensor | None = None, nsplit: int = 0,
                  bias: torch.Tensor | None = None, out_bf16: torch.Tensor | None = None, want_out: bool = True,
                  store_normed: bool = False, out_fp8: torch.Tensor | None = None,
                  out_fp8_scale: torch.Tensor | None = None):
    """v = x + bias + sum(parts[:nsplit]); x <- v (or LN(v) when ``store_normed``: post-LN models);
    out = bf16(LN(v)); optionally also the row-scaled e4m3 copy (``out_fp8`` + ``out_fp8_scale``)
    that feeds an fp8 GEMM.  parts: f32 [S, >=M, >=D]."""
    _req(x, torch.float32, "x", 2)
    M, D = x.shape
    if D % 4 or D > 2048 or gamma.numel() != D or beta.numel() != D:
        raise ValueError("add_layernorm: bad D/gamma/beta")
    ldp, sstride = 0, 0
    if nsplit:
        _req(parts, torch.float32, "parts", 3)
        if parts.shape[0] < nsplit or parts.shape[1] < M or parts.shape[2] < D:
            raise ValueError("add_layernorm: parts too small")
        ldp, sstride = parts.stride(1), parts.stride(0)
    if bias is not None:
        _req(bias, torch.float32, "bias", 1)
        if bias.numel() != D:
            raise ValueError("add_layernorm: bias size")
    if want_out and out_bf16 is None:
        out_bf16 = torch.empty(M, D, dtype=torch.bfloat16, device=x.device)
    if out_bf16 is not None:
        _req(out_bf16, torch.bfloat16, "out_bf16", 2)
        if out_bf16.shape[0] < M or out_bf16.shape[1] < D:
            raise ValueError("add_layernorm: out too small")
    ld8 = 0
    if out_fp8 is not None:
        _req(out_fp8, FP8, "out_fp8", 2)
        _req(out_fp8_scale, torch.float32, "out_fp8_scale", 1)
        if out_fp8.shape[0] < M or out_fp8.shape[1] < D or out_fp8_scale.numel() < M or out_fp8.stride(0) % 4:
            raise ValueError("add_layernorm: fp8 outputs too small / misaligned")
        ld8 = out_fp8.stride(0)
    _check(lib().dlms_add_layernorm(_p(x), x.stride(0), _p(parts) if nsplit else None, ldp, sstride, nsplit,
                                    _p(bias), _p(gamma), _p(beta), _p(out_bf16),
                                    out_bf16.stride(0) if out_bf16 is not None else 0, _p(out_fp8), ld8,
                                    _p(out_fp8_scale), M, D, float(eps), int(store_normed), _stream()),
           "dlms_add_layernorm")
    return out_bf16


def layernorm_gather(x: torch.Tensor, rows: torch.Tensor, gamma, beta, eps: float, out_bf16=None):
    _req(x, torch.float32, "x", 2)
    _req(rows, torch.int32, "rows", 1)
    M, D = rows.numel(), x.shape[1]
    if out_bf16 is None:
        out_bf16 = torch.empty(M, D, dtype=torch.bfloat16, device=x.device)
    _req(out_bf16, torch.bfloat16, "out_bf16", 2)
    if D % 4 or D > 2048 or gamma.numel() != D:
        raise ValueError("layernorm_gather: bad D")
    _check(lib().dlms_layernorm_gather(_p(x), x.stride(0), _p(rows), _p(gamma), _p(beta), _p(out_bf16),
                                       out_bf16.stride(0), M, D, float(eps), _stream()), "dlms_layernorm_gather")
    return out_bf16


def row_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, row_slot: torch.Tensor,
                  row_kvlen: torch.Tensor, out: torch.Tensor | None = None, scale: float | None = None,
                  impl: str = "wave", blocks: int = 512):
    """q: bf16 [R, H*64]; caches bf16 [slots, H, t_max, 64]; row r attends keys [0, row_kvlen[r]).
    impl "wave": one wave per (row, head), online softmax (default); "lds": block per (row, head),
    exact two-pass softmax through LDS (t_max <= 2048)."""
    _req(q, torch.bfloat16, "q", 2)
    _req(k_cache, torch.bfloat16, "k_cache", 4)
    _req(v_cache, torch.bfloat16, "v_cache", 4)
    _req(row_slot, torch.int32, "row_slot", 1)
    _req(row_kvlen, torch.int32, "row_kvlen", 1)
    R = q.shape[0]
    S, H, T, hd = k_cache.shape
    if hd != 64 or v_cache.shape != k_cache.shape or q.shape[1] < H * 64 or T > 2048:
        raise ValueError("row_attention: bad shapes")
    if row_slot.numel() < R or row_kvlen.numel() < R:
        raise ValueError("row_attention: index arrays too short")
    if out is None:
        out = torch.empty(R, H * 64, dtype=torch.bfloat16, device=q.device)
    _req(out, torch.bfloat16, "out", 2)
    sc = (1.0 / 8.0) if scale is None else scale
    if impl == "persist":  # fixed low-occupancy grid looping over (row, head) pairs
        _check(lib().dlms_attention_persist(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(row_slot), _p(row_kvlen),
                                            _p(out), out.stride(0), R, H, T, S, float(sc), int(blocks), _stream()),
               "attention_persist")
        return out
    fn = lib().dlms_attention if impl == "wave" else lib().dlms_row_attention
    _check(fn(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(row_slot), _p(row_kvlen), _p(out), out.stride(0), R, H,
              T, S, float(sc), _stream()), "attention")
    return out


class AttnTiles:
    """16-query tiles of packed sequences for ``tile_attention``: int32 [ntiles, 2] (row0, nq) on
    the device, plus the host-known number of packed rows they cover (checked against ``q``)."""

    def __init__(self, lens, device):
        import numpy as np

        lens = np.asarray(list(lens), dtype=np.int64)
        if lens.size == 0 or lens.min() < 1:
            raise ValueError("AttnTiles: every sequence needs >= 1 row")
        nt = (lens + 15) // 16
        starts = np.cumsum(lens) - lens
        seq = np.repeat(np.arange(lens.size), nt)
        k = np.arange(int(nt.sum())) - np.repeat(np.cumsum(nt) - nt, nt)
        row0 = starts[seq] + 16 * k
        nq = np.minimum(16, lens[seq] - 16 * k)
        self.rows = int(lens.sum())
        self.n = int(nt.sum())
        t = torch.from_numpy(np.stack([row0, nq], axis=1).astype(np.int32))
        if torch.device(device).type == "cuda":
            t = t.pin_memory()  # a pageable copy would block the host until the GPU reaches it
        self.t = t.to(device, non_blocking=True)


def tile_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, row_slot: torch.Tensor,
                   row_kvlen: torch.Tensor, tiles: AttnTiles, out: torch.Tensor | None = None,
                   scale: float | None = None):
    """MFMA attention over 16-query tiles (prefill / encoder): same contract as ``row_attention``
    (row r attends keys [0, row_kvlen[r]) of slot row_slot[r]); every tile's rows belong to one
    sequence (``AttnTiles`` builds them from the packed sequence lengths)."""
    _req(q, torch.bfloat16, "q", 2)
    _req(k_cache, torch.bfloat16, "k_cache", 4)
    _req(v_cache, torch.bfloat16, "v_cache", 4)
    _req(row_slot, torch.int32, "row_slot", 1)
    _req(row_kvlen, torch.int32, "row_kvlen", 1)
    R = q.shape[0]
    S, H, T, hd = k_cache.shape
    if hd != 64 or v_cache.shape != k_cache.shape or q.shape[1] < H * 64:
        raise ValueError("tile_attention: bad shapes")
    if not k_cache.is_contiguous() or not v_cache.is_contiguous():
        raise ValueError("tile_attention: caches must be contiguous")
    if tiles.rows > R or row_slot.numel() < tiles.rows or row_kvlen.numel() < tiles.rows:
        raise ValueError("tile_attention: tiles cover more rows than q / index arrays hold")
    if out is None:
        out = torch.empty(R, H * 64, dtype=torch.bfloat16, device=q.device)
    _req(out, torch.bfloat16, "out", 2)
    if out.shape[0] < tiles.rows or q.stride(0) % 8 or out.stride(0) % 8 or q.data_ptr() % 16 or out.data_ptr() % 16:
        raise ValueError("tile_attention: rows must be 16-byte aligned")
    sc = (1.0 / 8.0) if scale is None else scale
    _check(lib().dlms_tile_attention(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(row_slot), _p(row_kvlen),
                                     _p(tiles.t), tiles.n, _p(out), out.stride(0), H, T, k_cache.shape[0], float(sc),
                                     _stream()),
           "tile_attention")
    return out


def embed(tokens: torch.Tensor, positions: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor, out=None):
    _req(tokens, torch.int32, "tokens", 1)
    _req(positions, torch.int32, "positions", 1)
    _req(wte, torch.bfloat16, "wte", 2)
    _req(wpe, torch.bfloat16, "wpe", 2)
    R, D = tokens.numel(), wte.shape[1]
    if out is None:
        out = torch.empty(R, D, dtype=torch.float32, device=tokens.device)
    _req(out, torch.float32, "out", 2)
    _check(lib().dlms_embed(_p(tokens), _p(positions), _p(wte), _p(wpe), _p(out), out.stride(0), R, D, wte.shape[0],
                            wpe.shape[0], _stream()),
           "dlms_embed")
    return out


def argmax_reduce(parts: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """[B, P] partial argmax keys -> [B] (max per row)."""
    _req(parts, torch.int64, "parts", 2)
    B, P = parts.shape
    if out is None:
        out = torch.empty(B, dtype=torch.int64, device=parts.device)
    _req(out, torch.int64, "out", 1)
    if out.numel() < B:
        raise ValueError("argmax_reduce: out too short")
    _check(lib().dlms_argmax_reduce(_p(parts), P, parts.stride(0), _p(out), B, _stream()), "dlms_argmax_reduce")
    return out


def seen_set(seen: torch.Tensor, rows: torch.Tensor, tokens: torch.Tensor):
    """OR the bit of every ``tokens[i]`` into ``seen[rows[i]]`` (int32 bitmap rows of V/32 words).
    Callers validate rows (< seen.shape[0]) and ids on the host before upload; the kernel also skips
    ids outside [0, 32 * words)."""
    _req(seen, torch.int32, "seen", 2)
    _req(rows, torch.int32, "rows", 1)
    _req(tokens, torch.int32, "tokens", 1)
    R = tokens.numel()
    if rows.numel() != R or not seen.is_contiguous():
        raise ValueError("seen_set: one row per token, contiguous bitmap")
    if R == 0:
        return seen
    _check(lib().dlms_seen_set(_p(tokens), _p(rows), R, _p(seen), seen.shape[1], seen.shape[0], _stream()),
           "dlms_seen_set")
    return seen


def decode_update(keys: torch.Tensor, lens, finished, out_tokens, seen, cur_tok, cur_pos, cur_kvlen, wte, wpe, x,
                  eos: int, t_max: int, slot_map: torch.Tensor | None = None, ln=None, h: torch.Tensor | None = None):
    """keys: int64 [R, P] (row-major partial keys) or a transposed view [P, R].T (gathered per-rank
    keys); the token of row i is the argmax over its P keys and updates sequence slot
    ``slot_map[i]`` (default: slot i).  ``ln=(gamma, beta, eps)`` + ``h``: also write
    bf16(LN(x_new) * gamma + beta) of every updated slot into ``h`` (layer 0's LN1, bit-identical to
    ``add_layernorm`` on the stored row)."""
    if keys.dtype != torch.int64 or keys.device.type != "cuda" or keys.dim() != 2:
        raise ValueError("decode_update: keys must be a 2-D int64 GPU tensor")
    B, P = keys.shape
    nslots = B
    if slot_map is not None:
        _req(slot_map, torch.int32, "slot_map", 1)
        if slot_map.numel() < B:
            raise ValueError("slot_map too short")
        nslots = lens.numel()  # callers guarantee every slot_map entry is < the state capacity
    for t, n in ((lens, "lens"), (finished, "finished"), (cur_tok, "cur_tok"), (cur_pos, "cur_pos"),
                 (cur_kvlen, "cur_kvlen")):
        _req(t, torch.int32, n, 1)
        if t.numel() < nslots:
            raise ValueError(f"{n} too short")
    _req(out_tokens, torch.int32, "out_tokens", 2)
    _req(seen, torch.int32, "seen", 2)
    _req(x, torch.float32, "x", 2)
    D = wte.shape[1]
    if out_tokens.shape[0] < nslots or x.shape[0] < nslots or x.shape[1] < D or seen.shape[0] < nslots:
        raise ValueError("decode_update: buffers too small")
    g = b = None
    eps = 0.0
    if (ln is None) != (h is None):
        raise ValueError("decode_update: ln and h go together")
    if h is not None:
        g, b, eps = ln
        _req(h, torch.bfloat16, "h", 2)
        for t, n in ((g, "gamma"), (b, "beta")):
            _req(t, torch.float32, n, 1)
            if t.numel() < D or not t.is_contiguous():
                raise ValueError(f"decode_update: {n} must be contiguous [D]")
        if h.shape[0] < nslots or h.shape[1] < D or h.stride(1) != 1 or h.stride(0) % 4 or h.data_ptr() % 8:
            raise ValueError("decode_update: h must be [>= slots, >= D] bf16 rows, 8-B aligned")
    _check(lib().dlms_decode_update(_p(keys), P, keys.stride(0), keys.stride(1), _p(slot_map), _p(lens), _p(finished),
                                    _p(out_tokens),
                                    out_tokens.stride(0), _p(seen), seen.stride(0), _p(cur_tok), _p(cur_pos),
                                    _p(cur_kvlen), _p(wte), _p(wpe), _p(x), x.stride(0), B, D, eos, t_max,
                                    lens.numel(), wte.shape[0], _p(g), _p(b), float(eps), _p(h),
                                    h.stride(0) if h is not None else 0, _stream()),
           "dlms_decode_update")


def bert_embed_ln(ids, positions, word, pos_emb, type0, gamma, beta, eps: float, out_f32=None, out_bf16=None):
    _req(ids, torch.int32, "ids", 1)
    _req(positions, torch.int32, "positions", 1)
    for t, n in ((word, "word"), (pos_emb, "pos_emb")):
        _req(t, torch.float32, n, 2)
    R, D = ids.numel(), word.shape[1]
    if out_f32 is None:
        out_f32 = torch.empty(R, D, dtype=torch.float32, device=ids.device)
    if out_bf16 is None:
        out_bf16 = torch.empty(R, D, dtype=torch.bfloat16, device=ids.device)
    _check(lib().dlms_bert_embed_ln(_p(ids), _p(positions), _p(word), _p(pos_emb), _p(type0), _p(gamma), _p(beta),
                                    _p(out_f32), _p(out_bf16), R, D, float(eps), word.shape[0], pos_emb.shape[0],
                                    _stream()), "dlms_bert_embed_ln")
    return out_f32, out_bf16


def mean_pool(x: torch.Tensor, start: torch.Tensor, length: torch.Tensor, out=None):
    _req(x, torch.float32, "x", 2)
    _req(start, torch.int32, "start", 1)
    _req(length, torch.int32, "length", 1)
    S, D = start.numel(), x.shape[1]
    if not x.is_contiguous():
        raise ValueError("mean_pool: x must be contiguous")
    if out is None:
        out = torch.empty(S, D, dtype=torch.float32, device=x.device)
    _check(lib().dlms_mean_pool(_p(x), _p(start), _p(length), _p(out), S, D, _stream()), "dlms_mean_pool")
    return out


def cosine(a: torch.Tensor, b: torch.Tensor, eps: float = 1e-8, out=None):
    _req(a, torch.float32, "a", 2)
    _req(b, torch.float32, "b", 2)
    if a.shape[1] != b.shape[1] or not a.is_contiguous() or not b.is_contiguous():
        raise ValueError("cosine: bad shapes")
    if out is None:
        out = torch.empty(a.shape[0], b.shape[0], dtype=torch.float32, device=a.device)
    _check(lib().dlms_cosine(_p(a), _p(b), _p(out), a.shape[0], b.shape[0], a.shape[1], float(eps), _stream()),
           "dlms_cosine")
    return out


# ---------------------------------------------------------------------------------------------
# Skinny (M <= 32) decode GEMMs on pre-shuffled weights + split-K flash-decode (skinny.hip)
# ---------------------------------------------------------------------------------------------
SKINNY_MAX_M = 32


def shuffle_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] bf16 (K contiguous) -> MFMA B-fragment order [N/16, K/32, 64, 8]: lane l of the
    16x16x32 bf16 MFMA holds W[16 ng + (l & 15)][32 kb + 8 (l >> 4) + j] at [ng, kb, l, j], so one
    contiguous KiB per (column group, k-block) is one wave-load straight into the B operand."""
    if w.dim() != 2 or w.shape[0] % 16 or w.shape[1] % 32:
        raise ValueError(f"shuffle_weight: need [N%16, K%32], got {tuple(w.shape)}")
    N, K = w.shape
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(N // 16, K // 32, 64, 8).contiguous()


def unshuffle_weight(ws: torch.Tensor) -> torch.Tensor:
    """Inverse of ``shuffle_weight`` (tests)."""
    G, KB = ws.shape[0], ws.shape[1]
    return ws.reshape(G, KB, 4, 16, 8).permute(0, 3, 1, 2, 4).reshape(G * 16, KB * 32)


def _skinny_epi(a: torch.Tensor, M: int, N: int, epi: int, bias, out, q_out, k_cache, v_cache, row_slot, row_pos,
                argmax_out, seen, vocab: int, col_offset: int, penalty: float, name: str = "skinny_gemm"):
    """GemmEpi of the skinny / mid kernels' column-owning epilogue (skinny_common.h): returns
    (ep, kernel epilogue id, output tensor)."""
    ep = GemmEpi()
    if bias is not None:
        _req(bias, torch.float32, "bias", 1)
        if bias.numel() < N:
            raise ValueError("bias too short")
        ep.bias = bias.data_ptr()
    cepi = epi
    if epi == EPI_F32 and out is not None and out.dtype == torch.int64:
        cepi = 7  # skinny.hip SK_FIXADD: into copy 0 of the fused MLP's fixed-point residual
    if epi in (EPI_BF16, EPI_GELU_TANH, EPI_F32, EPI_PARTIAL):
        want = torch.bfloat16 if epi in (EPI_BF16, EPI_GELU_TANH) else torch.float32
        if cepi == 7:
            want = torch.int64
        if out is None:
            if epi == EPI_F32:
                raise ValueError(f"{name} EPI_F32 accumulates into an existing out (the residual)")
            out = torch.empty(M, N, dtype=want, device=a.device)
        _req(out, want, "out", 2)
        if out.shape[0] < M or out.shape[1] < N:
            raise ValueError("out too small")
        ep.out, ep.ldo = out.data_ptr(), out.stride(0)
    elif epi == EPI_QKV:
        for t, n in ((q_out, "q_out"), (k_cache, "k_cache"), (v_cache, "v_cache")):
            _req(t, torch.bfloat16, n)
        _req(row_slot, torch.int32, "row_slot", 1)
        _req(row_pos, torch.int32, "row_pos", 1)
        if N % 3 or (N // 3) % 64:
            raise ValueError("QKV N must be 3 * d_local (64-wide heads)")
        d_local = N // 3
        if k_cache.dim() != 4 or k_cache.shape != v_cache.shape or k_cache.shape[1] * 64 != d_local or \
                k_cache.shape[3] != 64 or not k_cache.is_contiguous() or not v_cache.is_contiguous():
            raise ValueError(f"cache shape {tuple(k_cache.shape)} incompatible with d_local={d_local}")
        if q_out.shape[0] < M or q_out.shape[1] < d_local or row_slot.numel() < M or row_pos.numel() < M:
            raise ValueError("qkv epilogue buffers too small")
        ep.q_out, ep.ldq = q_out.data_ptr(), q_out.stride(0)
        ep.k_cache, ep.v_cache = k_cache.data_ptr(), v_cache.data_ptr()
        ep.row_slot, ep.row_pos = row_slot.data_ptr(), row_pos.data_ptr()
        ep.n_heads, ep.t_max, ep.d_local, ep.n_slots = k_cache.shape[1], k_cache.shape[2], d_local, k_cache.shape[0]
        out = q_out
    elif epi == EPI_ARGMAX:
        _req(argmax_out, torch.int64, "argmax_out", 2)
        _req(seen, torch.int32, "seen", 2)
        if N % 64 or argmax_out.shape[0] < M or argmax_out.shape[1] < N // 64 or seen.shape[0] < M or \
                seen.shape[1] * 32 < vocab or col_offset % 64:
            raise ValueError("argmax epilogue buffers too small / misaligned shard")
        ep.argmax_out, ep.ldo, ep.seen = argmax_out.data_ptr(), argmax_out.stride(0), seen.data_ptr()
        ep.seen_words, ep.vocab, ep.col_offset, ep.penalty = seen.stride(0), vocab, col_offset, penalty
        out = argmax_out
    else:
        raise ValueError(f"{name}: unsupported epilogue {epi}")
    return ep, cepi, out


def skinny_gemm(a: torch.Tensor, w_sh: torch.Tensor, epi: int, *, ln=None, bias=None, out=None,
                q_out=None, k_cache=None, v_cache=None, row_slot=None, row_pos=None,
                argmax_out=None, seen=None, vocab: int = 0, col_offset: int = 0, penalty: float = 1.0):
    """Decode GEMM for M <= 32 rows against a ``shuffle_weight`` weight ([N/16, K/32, 64, 8]).

    ``ln=(gamma, beta, eps)``: ``a`` is the f32 residual x [M, K] and the kernel LayerNorms it in
    its prologue (EPI_BF16 / EPI_GELU_TANH / EPI_QKV / EPI_ARGMAX: ln_f fused into the LM head);
    otherwise ``a`` is bf16 [M, K].
    EPI_F32 adds ``acc + bias`` into ``out`` (f32 [M, N], in place: the residual stream; an int64
    ``out`` is copy 0 of ``skinny_mlp``'s fixed-point residual and gets fix(acc + bias) added);
    EPI_PARTIAL stores the raw f32 partial (TP); EPI_ARGMAX writes one key per (row, 64 columns)
    into ``argmax_out`` [M, >= N/64] exactly like ``gemm(..., EPI_ARGMAX)``."""
    _req(w_sh, torch.bfloat16, "w_sh", 4)
    G, KB = w_sh.shape[0], w_sh.shape[1]
    if w_sh.shape[2] != 64 or w_sh.shape[3] != 8 or not w_sh.is_contiguous():
        raise ValueError("skinny_gemm: w_sh must be a contiguous shuffle_weight() tensor")
    N, K = G * 16, KB * 32
    if ln is not None:
        _req(a, torch.float32, "a", 2)
        g_, b_, eps = ln
        _req(g_, torch.float32, "ln gamma", 1)
        _req(b_, torch.float32, "ln beta", 1)
        if g_.numel() != K or b_.numel() != K or K > 2048 or K % 4:
            raise ValueError("skinny_gemm: LN params must match K (<= 2048)")
        if epi not in (EPI_BF16, EPI_GELU_TANH, EPI_QKV, EPI_ARGMAX):
            raise ValueError("skinny_gemm: the LayerNorm prologue feeds bf16 / GELU / QKV / argmax epilogues only")
    else:
        _req(a, torch.bfloat16, "a", 2)
        if epi in (EPI_GELU_TANH, EPI_QKV):
            raise ValueError("skinny_gemm: GELU / QKV epilogues take the LN prologue")
        if a.stride(0) % 8 or a.data_ptr() % 16:
            raise ValueError("skinny_gemm: bf16 A rows must be 16-byte aligned")
    M = a.shape[0]
    if a.shape[1] != K:
        raise ValueError(f"skinny_gemm: a has K={a.shape[1]}, weight K={K}")
    if M < 1 or M > SKINNY_MAX_M:
        raise ValueError(f"skinny_gemm: 1 <= M <= {SKINNY_MAX_M}")
    ep, cepi, out = _skinny_epi(a, M, N, epi, bias, out, q_out, k_cache, v_cache, row_slot, row_pos, argmax_out, seen,
                                vocab, col_offset, penalty)
    lg, lb, le = (ln[0], ln[1], float(ln[2])) if ln is not None else (None, None, 0.0)
    _check(lib().dlms_skinny_gemm(cepi, _p(a), a.stride(0), _p(lg), _p(lb), le, _p(w_sh), M, N, K, ctypes.byref(ep),
                                  _stream()), "dlms_skinny_gemm")
    return out


def cu_masked_stream(n_cus: int) -> "torch.cuda.ExternalStream":
    """A stream of the current device restricted to ``n_cus`` evenly spread compute units
    (``hipExtStreamCreateWithCUMask``, api.hip): co-located work that must not hold the CUs a
    latency-bound decode needs (the relevance gate beside the tutor)."""
    p = ctypes.c_void_p()
    _check(lib().dlms_stream_create_cumask(int(n_cus), ctypes.byref(p)), "dlms_stream_create_cumask")
    return torch.cuda.ExternalStream(p.value)


def mid_max_rows(K: int) -> int:
    """Largest M the mid-batch fused LayerNorm + GEMM (``mid_ln_gemm``) takes at width K (0: none)."""
    return int(lib().dlms_mid_max_rows(int(K)))


def mid_ln_gemm(x: torch.Tensor, w_sh: torch.Tensor, epi: int, gamma, beta, eps: float, *, bias=None, out=None,
                q_out=None, k_cache=None, v_cache=None, row_slot=None, row_pos=None, geo: int = 0):
    """Mid-batch decode (9-64 rows) LN1 -> QKV / LN2 -> c_fc in one kernel (mid.hip):
    ``out = epi(bf16(LN(x)) @ W.T + bias)`` for the f32 residual rows ``x`` [M, K] (complete: the
    mid path's projections update the residual in place) against a ``shuffle_weight`` weight.
    epi: EPI_QKV (q out + K/V cache scatter), EPI_GELU_TANH or EPI_BF16 (bf16 ``out``).
    ``geo``: 0 = default geometry, 1..5 tuning overrides (waves / column groups per workgroup)."""
    _req(x, torch.float32, "x", 2)
    _req(w_sh, torch.bfloat16, "w_sh", 4)
    G, KB = w_sh.shape[0], w_sh.shape[1]
    if w_sh.shape[2] != 64 or w_sh.shape[3] != 8 or not w_sh.is_contiguous():
        raise ValueError("mid_ln_gemm: w_sh must be a contiguous shuffle_weight() tensor")
    N, K = G * 16, KB * 32
    M = x.shape[0]
    if x.shape[1] != K or M < 1 or M > mid_max_rows(K) or x.stride(0) % 4 or x.data_ptr() % 16:
        raise ValueError(f"mid_ln_gemm: x {tuple(x.shape)} vs K={K} (max rows {mid_max_rows(K)}, 16-B aligned rows)")
    for t, n in ((gamma, "gamma"), (beta, "beta")):
        _req(t, torch.float32, n, 1)
        if t.numel() != K:
            raise ValueError(f"mid_ln_gemm: {n} size")
    if epi not in (EPI_QKV, EPI_GELU_TANH, EPI_BF16):
        raise ValueError("mid_ln_gemm: QKV / GELU / bf16 epilogues")
    ep, cepi, out = _skinny_epi(x, M, N, epi, bias, out, q_out, k_cache, v_cache, row_slot, row_pos, None, None, 0, 0,
                                1.0, name="mid_ln_gemm")
    _check(lib().dlms_mid_ln_gemm(cepi, _p(x), x.stride(0), _p(gamma), _p(beta), float(eps), _p(w_sh), M, N, K,
                                  ctypes.byref(ep), int(geo), _stream()), "dlms_mid_ln_gemm")
    return out


def mid_proj(a: torch.Tensor, w_sh: torch.Tensor, x: torch.Tensor, *, bias=None, geo: int = 0) -> torch.Tensor:
    """Mid-batch (<= 64 rows) in-place row-parallel projection (mid.hip): ``x += a @ W.T + bias``
    with column-owning workgroups (out-projection, c_proj).  a: bf16 [M, K]; x: f32 [M, N];
    ``w_sh``: ``shuffle_weight`` layout.  K/32 must split evenly over the geometry's waves."""
    _req(a, torch.bfloat16, "a", 2)
    _req(x, torch.float32, "x", 2)
    _req(w_sh, torch.bfloat16, "w_sh", 4)
    G, KB = w_sh.shape[0], w_sh.shape[1]
    if w_sh.shape[2] != 64 or w_sh.shape[3] != 8 or not w_sh.is_contiguous():
        raise ValueError("mid_proj: w_sh must be a contiguous shuffle_weight() tensor")
    N, K = G * 16, KB * 32
    M = a.shape[0]
    if a.shape[1] != K or x.shape[0] != M or x.shape[1] != N or not 1 <= M <= 64:
        raise ValueError(f"mid_proj: a {tuple(a.shape)}, x {tuple(x.shape)} vs W [{N}, {K}] (1 <= M <= 64)")
    if a.stride(0) % 8 or a.data_ptr() % 16:
        raise ValueError("mid_proj: bf16 A rows must be 16-byte aligned")
    if bias is not None:
        _req(bias, torch.float32, "bias", 1)
        if bias.numel() < N:
            raise ValueError("mid_proj: bias too short")
    _check(lib().dlms_mid_proj(_p(a), a.stride(0), _p(w_sh), _p(bias), _p(x), x.stride(0), M, N, K, int(geo),
                               _stream()), "dlms_mid_proj")
    return x


def skinny_addln_max_rows(K: int) -> int:
    """Largest M the fused add+LN skinny GEMM takes at model width K (0 = unsupported)."""
    return int(lib().dlms_skinny_addln_max_rows(int(K)))


def skinny_addln_gemm(x_in: torch.Tensor, w_sh: torch.Tensor, epi: int, gamma, beta, eps: float, *, x_out=None,
                      parts=None, nsplit: int = 0, res_bias=None, bias=None, out=None, q_out=None, k_cache=None,
                      v_cache=None, row_slot=None, row_pos=None, zero=None):
    """Fused residual update + LayerNorm + skinny GEMM (decode LN1 -> QKV, LN2 -> c_fc) for
    M <= ``skinny_addln_max_rows(K)`` rows:

        v = x_in + res_bias + sum(parts[:nsplit]);  x_out <- v (when given);
        out = epi(bf16(LN(v)) @ W.T + bias)

    ``x_out`` must not alias ``x_in`` (every workgroup re-reads x_in; one of them writes x_out):
    the engine ping-pongs two residual buffers.  nsplit in {0, 1, 4}, or 12 / 16 (per-head slabs of
    ``attention_oproj``; M <= 4, K <= 1024).

    ``x_in`` may be the int64 fixed-point residual a ``skinny_mlp`` left ([FIX_COPIES, M, K]; QKV
    epilogue, no slabs, no x_out); ``zero``: a contiguous tensor (the next ``skinny_mlp``'s
    accumulator) the kernel clears on the side."""
    xfix = x_in.dtype == torch.int64
    xcs = 0
    if xfix:
        if epi != EPI_QKV or nsplit or x_out is not None:
            raise ValueError("skinny_addln_gemm: a fixed-point residual feeds only the QKV epilogue, no slabs")
        _req(x_in, torch.int64, "x_in", 3)
        if x_in.shape[0] != fix_copies() or x_in.stride(0) % 2:
            raise ValueError(f"skinny_addln_gemm: fixed-point x_in must be [{fix_copies()}, M, K]")
        xcs = x_in.stride(0)
        x_in = x_in[0]
    else:
        _req(x_in, torch.float32, "x_in", 2)
    zchunks = 0
    if zero is not None:
        if not zero.is_contiguous() or zero.data_ptr() % 16 or (zero.numel() * zero.element_size()) % 16:
            raise ValueError("skinny_addln_gemm: zero must be a contiguous 16-byte multiple")
        if zero.data_ptr() == x_in.data_ptr():
            raise ValueError("skinny_addln_gemm: zero must not alias x_in")
        zchunks = zero.numel() * zero.element_size() // 16
    _req(w_sh, torch.bfloat16, "w_sh", 4)
    G, KB = w_sh.shape[0], w_sh.shape[1]
    if w_sh.shape[2] != 64 or w_sh.shape[3] != 8 or not w_sh.is_contiguous():
        raise ValueError("skinny_addln_gemm: w_sh must be a contiguous shuffle_weight() tensor")
    N, K = G * 16, KB * 32
    M = x_in.shape[0]
    if x_in.shape[1] != K or M < 1 or M > skinny_addln_max_rows(K):
        raise ValueError(f"skinny_addln_gemm: x_in {tuple(x_in.shape)} vs K={K}, max rows {skinny_addln_max_rows(K)}")
    for t, n in ((gamma, "gamma"), (beta, "beta")):
        _req(t, torch.float32, n, 1)
        if t.numel() != K:
            raise ValueError(f"{n} size")
    if nsplit not in (0, 1, 4, 12, 16):
        raise ValueError("skinny_addln_gemm: nsplit in {0, 1, 4, 12, 16}")
    if nsplit > 4 and (x_in.shape[0] > 4 or x_in.shape[1] > 1024):
        raise ValueError("skinny_addln_gemm: 12/16 slabs only for <= 4 rows of width <= 1024")
    ldp, sstride = 0, 0
    if nsplit:
        _req(parts, torch.float32, "parts", 3)
        if parts.shape[0] < nsplit or parts.shape[1] < M or parts.shape[2] < K or parts.stride(1) % 4 or \
                parts.stride(0) % 4:
            raise ValueError("skinny_addln_gemm: parts too small / misaligned")
        ldp, sstride = parts.stride(1), parts.stride(0)
    if res_bias is not None:
        _req(res_bias, torch.float32, "res_bias", 1)
        if res_bias.numel() != K:
            raise ValueError("res_bias size")
    if x_out is not None:
        _req(x_out, torch.float32, "x_out", 2)
        if x_out.shape[0] < M or x_out.shape[1] < K or x_out.stride(0) != x_in.stride(0):
            raise ValueError("skinny_addln_gemm: x_out must match x_in's layout")
        if x_out.data_ptr() == x_in.data_ptr():
            raise ValueError("skinny_addln_gemm: x_out must not alias x_in (ping-pong the residual)")
    if x_in.stride(0) % 4 or x_in.data_ptr() % 16 or not x_in.stride(1) == 1:
        raise ValueError("skinny_addln_gemm: x rows must be 16-byte aligned")
    ep = GemmEpi()
    if bias is not None:
        _req(bias, torch.float32, "bias", 1)
        if bias.numel() < N:
            raise ValueError("bias too short")
        ep.bias = bias.data_ptr()
    if epi == EPI_GELU_TANH:
        if out is None:
            out = torch.empty(M, N, dtype=torch.bfloat16, device=x_in.device)
        _req(out, torch.bfloat16, "out", 2)
        if out.shape[0] < M or out.shape[1] < N:
            raise ValueError("out too small")
        ep.out, ep.ldo = out.data_ptr(), out.stride(0)
    elif epi == EPI_QKV:
        for t, n in ((q_out, "q_out"), (k_cache, "k_cache"), (v_cache, "v_cache")):
            _req(t, torch.bfloat16, n)
        _req(row_slot, torch.int32, "row_slot", 1)
        _req(row_pos, torch.int32, "row_pos", 1)
        if N % 3 or (N // 3) % 64:
            raise ValueError("QKV N must be 3 * d_local (64-wide heads)")
        d_local = N // 3
        if k_cache.dim() != 4 or k_cache.shape != v_cache.shape or k_cache.shape[1] * 64 != d_local or \
                k_cache.shape[3] != 64 or not k_cache.is_contiguous() or not v_cache.is_contiguous():
            raise ValueError(f"cache shape {tuple(k_cache.shape)} incompatible with d_local={d_local}")
        if q_out.shape[0] < M or q_out.shape[1] < d_local or row_slot.numel() < M or row_pos.numel() < M:
            raise ValueError("qkv epilogue buffers too small")
        ep.q_out, ep.ldq = q_out.data_ptr(), q_out.stride(0)
        ep.k_cache, ep.v_cache = k_cache.data_ptr(), v_cache.data_ptr()
        ep.row_slot, ep.row_pos = row_slot.data_ptr(), row_pos.data_ptr()
        ep.n_heads, ep.t_max, ep.d_local, ep.n_slots = k_cache.shape[1], k_cache.shape[2], d_local, k_cache.shape[0]
        out = q_out
    else:
        raise ValueError("skinny_addln_gemm: QKV or GELU epilogue")
    _check(lib().dlms_skinny_addln_gemm(epi, _p(x_in), _p(x_out), x_in.stride(0), _p(parts) if nsplit else None, ldp,
                                        sstride, nsplit, _p(res_bias), _p(gamma), _p(beta), float(eps), _p(w_sh), M, N,
                                        K, ctypes.byref(ep), int(xfix), xcs, _p(zero), zchunks, _stream()),
           "dlms_skinny_addln_gemm")
    return out


def slice_cproj(w_p: torch.Tensor) -> torch.Tensor:
    """c_proj weight [d, F] (F = 4d contiguous) -> [F/16, d, 16]: the contiguous 16-column slab each
    ``skinny_mlp`` workgroup streams."""
    if w_p.dim() != 2 or w_p.shape[1] % 16:
        raise ValueError(f"slice_cproj: need [d, F % 16], got {tuple(w_p.shape)}")
    d, F = w_p.shape
    return w_p.reshape(d, F // 16, 16).permute(1, 0, 2).contiguous()


FIX_SCALE = float(2 ** 32)  # skinny.hip DLMS_FIX_SCALE: the fused MLP's int64 fixed-point residual


def fix_copies() -> int:
    """Partial copies of the fixed-point residual ([fix_copies(), M, d]; readers sum them)."""
    return int(lib().dlms_fix_copies())


def fix_to_float(r: torch.Tensor) -> torch.Tensor:
    """int64 fixed-point residual [fix_copies(), M, d] -> f32 [M, d] (tests / debugging)."""
    return (r.sum(0).to(torch.float64) / FIX_SCALE).to(torch.float32)


SKINNY_MLP_WIDTHS = (768, 1024, 1280, 1600)  # GPT-2 small / medium / large / XL


def skinny_mlp_cg(K: int, M: int, want: int = 0) -> int:
    """Column groups per workgroup the fused MLP uses for M rows of width K (0: unsupported)."""
    return int(lib().dlms_skinny_mlp_cg(K, M, want))


def skinny_mlp(x_in: torch.Tensor, gamma, beta, eps: float, w_fc_sh: torch.Tensor, b_fc, w_p_sl: torch.Tensor, b_p,
               r_out: torch.Tensor, *, parts=None, nsplit: int = 0, res_bias=None, cg: int = 0, base: bool = True):
    """Fused latency-path MLP (M <= 8 rows, d in SKINNY_MLP_WIDTHS):

        v = x_in + res_bias + sum(parts[:nsplit]);  h = bf16(gelu(bf16(LN(v)) @ W_fc.T + b_fc))
        r_out += fix(v + h @ W_p.T + b_p)          (base=False: r_out += fix(h @ W_p.T) only)

    Tensor parallel (``W_fc`` / ``b_fc`` the rank's column shard, ``W_p`` its row-parallel slice,
    ``parts`` the all-reduced attention partial, nsplit 1): rank 0 runs with base=True, the others
    with base=False, and an integer all-reduce of ``r_out`` over the group is the next residual.

    ``x_in``: f32 [M, d] or int64 fixed point [fix_copies(), M, d]; ``r_out``: int64 fixed point
    [fix_copies(), M, d], ZERO on entry (``skinny_addln_gemm(zero=...)`` clears it), must not alias
    ``x_in``.  Workgroup j adds its contribution into copy j % fix_copies() with 64-bit integer
    atomics: the result is order-independent.  ``cg``: column groups of 16 intermediate columns
    per workgroup (1, 2, 4; 0 = DLMS_MLP_CG or the per-width default; narrowed to what fits the LDS)."""
    xfix = x_in.dtype == torch.int64
    C = fix_copies()
    xcs = 0
    if xfix:
        _req(x_in, torch.int64, "x_in", 3)
        if x_in.shape[0] != C or x_in.stride(0) % 2:
            raise ValueError(f"skinny_mlp: fixed-point x_in must be [{C}, M, d]")
        xcs = x_in.stride(0)
        x_in = x_in[0]
    else:
        _req(x_in, torch.float32, "x_in", 2)
    _req(r_out, torch.int64, "r_out", 3)
    if r_out.shape[0] != C or r_out.stride(0) % 2:
        raise ValueError(f"skinny_mlp: r_out must be [{C}, M, d]")
    rcs = r_out.stride(0)
    r_full, r_out = r_out, r_out[0]
    _req(w_fc_sh, torch.bfloat16, "w_fc_sh", 4)
    _req(w_p_sl, torch.bfloat16, "w_p_sl", 3)
    M, K = x_in.shape
    F = w_fc_sh.shape[0] * 16
    if w_fc_sh.shape[1] * 32 != K or not w_fc_sh.is_contiguous() or tuple(w_p_sl.shape) != (F // 16, K, 16) or \
            not w_p_sl.is_contiguous():
        raise ValueError("skinny_mlp: weight layouts (shuffle_weight / slice_cproj) do not match x_in")
    if M < 1 or M > 8 or K not in SKINNY_MLP_WIDTHS:
        raise ValueError(f"skinny_mlp: M <= 8 rows of width {SKINNY_MLP_WIDTHS}, got {tuple(x_in.shape)}")
    if skinny_mlp_cg(K, M, cg) == 0:
        raise ValueError(f"skinny_mlp: {M} rows of width {K} do not fit the kernel's LDS")
    if r_out.shape[0] < M or r_out.shape[1] < K or r_out.stride(1) != 1 or r_out.data_ptr() == x_in.data_ptr():
        raise ValueError("skinny_mlp: r_out too small or aliases x_in")
    if x_in.stride(1) != 1 or x_in.stride(0) % 4 or x_in.data_ptr() % 16:
        raise ValueError("skinny_mlp: x rows must be 16-byte aligned")
    for t, n, size in ((gamma, "gamma", K), (beta, "beta", K), (b_fc, "b_fc", F), (b_p, "b_p", K)):
        _req(t, torch.float32, n, 1)
        if t.numel() != size:
            raise ValueError(f"skinny_mlp: {n} size")
    if nsplit not in (0, 1, 4) or (nsplit == 4 and K > 1024):
        raise ValueError("skinny_mlp: nsplit in {0, 1, 4} (4: d <= 1024)")
    ldp, sstride = 0, 0
    if nsplit:
        _req(parts, torch.float32, "parts", 3)
        if parts.shape[0] < nsplit or parts.shape[1] < M or parts.shape[2] < K or parts.stride(2) != 1 or \
                parts.stride(1) % 4 or parts.stride(0) % 4:
            raise ValueError("skinny_mlp: parts too small / misaligned")
        ldp, sstride = parts.stride(1), parts.stride(0)
    if res_bias is not None:
        _req(res_bias, torch.float32, "res_bias", 1)
        if res_bias.numel() != K:
            raise ValueError("res_bias size")
    _check(lib().dlms_skinny_mlp(_p(x_in), x_in.stride(0), int(xfix), xcs, _p(parts) if nsplit else None, ldp,
                                 sstride, nsplit, _p(res_bias), _p(gamma), _p(beta), float(eps), _p(w_fc_sh), _p(b_fc),
                                 _p(w_p_sl), _p(b_p), _p(r_out), r_out.stride(0), rcs, M, K, F, int(cg), int(bool(base)),
                                 _stream()),
           "dlms_skinny_mlp")
    return r_full


def ln_fix(x: torch.Tensor, gamma, beta, eps: float, out: torch.Tensor):
    """LayerNorm of an int64 fixed-point residual [fix_copies(), M, K] -> bf16 ``out`` (ln_f after
    ``skinny_mlp``)."""
    _req(x, torch.int64, "x", 3)
    _req(out, torch.bfloat16, "out", 2)
    if x.shape[0] != fix_copies() or x.stride(0) % 2:
        raise ValueError(f"ln_fix: x must be [{fix_copies()}, M, K]")
    xcs, x = x.stride(0), x[0]
    M, K = x.shape
    if x.stride(1) != 1 or out.stride(1) != 1 or out.shape[0] < M or out.shape[1] < K or x.stride(0) % 2 or \
            out.stride(0) % 4 or K % 4 or K > 2048 or x.data_ptr() % 16 or out.data_ptr() % 8:
        raise ValueError("ln_fix: shapes / alignment")
    for t, n in ((gamma, "gamma"), (beta, "beta")):
        _req(t, torch.float32, n, 1)
        if t.numel() != K:
            raise ValueError(f"ln_fix: {n} size")
    _check(lib().dlms_ln_fix(_p(x), x.stride(0), xcs, _p(gamma), _p(beta), float(eps), _p(out), out.stride(0), M, K,
                             _stream()), "dlms_ln_fix")
    return out


def attention_split_waves(kv_len_max: int) -> int:
    """Waves per (row, head) for ``attention_split``: about 32 keys per wave, 2..16."""
    for nw in (2, 4, 8, 16):
        if kv_len_max <= 32 * nw:
            return nw
    return 16


ATTN_WS_STRIDE = 68  # floats per cross-workgroup partial (skinny.hip)
# publish mode of the cross-workgroup split attention: write-through partials + a vmcnt wait (0:
# __threadfence, 2x slower; 1: write-through + agent fences) -- profiles/r2_attn_splitwg.jsonl
ATTN_SPLIT_SYNC = 2


def attention_split_geometry(pairs: int, kv_len_max: int, cus: int = 256) -> tuple[int, int]:
    """(waves, workgroups) per (row, head) for ``attention_split``.  Splitting a pair's keys over
    several workgroups fills more CUs but adds two dependent global round trips (arrival atomic,
    partial reload) to the kernel's latency chain; measured on MI355X (profiles/r2_attn_splitwg.jsonl)
    that only pays for a handful of pairs with long caches (B=1, T=1024: 9.8 vs 11.1 us), and is
    neutral to slower from B=8 on -- there, one 16-wave workgroup per pair is kept."""
    nw = attention_split_waves(kv_len_max)
    if pairs <= 32 and kv_len_max > 512:
        return 8, 4
    return nw, 1


class AttnSplitWorkspace:
    """Partials + arrival counters for cross-workgroup ``attention_split`` (counters start at 0
    and every launch re-arms them, so one workspace serves every replay of a captured graph)."""

    def __init__(self, pairs: int, splits: int, device):
        self.pairs, self.splits = pairs, splits
        self.partials = torch.empty(pairs * splits * ATTN_WS_STRIDE, dtype=torch.float32, device=device)
        self.counters = torch.zeros(pairs, dtype=torch.int32, device=device)

    def fits(self, pairs: int, splits: int) -> bool:
        return pairs <= self.pairs and pairs * splits <= self.pairs * self.splits


def attention_split(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, row_slot: torch.Tensor,
                    row_kvlen: torch.Tensor, out: torch.Tensor | None = None, scale: float | None = None,
                    waves: int = 16, splits: int = 1, workspace: "AttnSplitWorkspace | None" = None,
                    sync: int | None = None):
    """Split-K flash-decode: ``splits`` workgroups of ``waves`` waves per (row, head), each wave
    streaming a slice of the keys; waves merge by log-sum-exp in LDS, workgroups through a
    workspace merged by the last to arrive.  Same contract as ``row_attention``."""
    _req(q, torch.bfloat16, "q", 2)
    _req(k_cache, torch.bfloat16, "k_cache", 4)
    _req(v_cache, torch.bfloat16, "v_cache", 4)
    _req(row_slot, torch.int32, "row_slot", 1)
    _req(row_kvlen, torch.int32, "row_kvlen", 1)
    R = q.shape[0]
    S, H, T, hd = k_cache.shape
    if hd != 64 or v_cache.shape != k_cache.shape or q.shape[1] < H * 64:
        raise ValueError("attention_split: bad shapes")
    if row_slot.numel() < R or row_kvlen.numel() < R:
        raise ValueError("attention_split: index arrays too short")
    if waves not in (2, 4, 8, 16):
        raise ValueError("attention_split: waves in {2, 4, 8, 16}")
    if not 1 <= splits <= 64:
        raise ValueError("attention_split: splits in [1, 64]")
    if out is None:
        out = torch.empty(R, H * 64, dtype=torch.bfloat16, device=q.device)
    _req(out, torch.bfloat16, "out", 2)
    ws_p = cnt_p = None
    if splits > 1:
        if workspace is None:
            workspace = AttnSplitWorkspace(R * H, splits, q.device)
        if not workspace.fits(R * H, splits):
            raise ValueError("attention_split: workspace too small")
        ws_p, cnt_p = _p(workspace.partials), _p(workspace.counters)
    sc = (1.0 / 8.0) if scale is None else scale
    _check(lib().dlms_attention_split(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(row_slot), _p(row_kvlen),
                                      _p(out), out.stride(0), R, H, T, S, float(sc), int(waves), int(splits),
                                      ws_p, cnt_p, ATTN_SPLIT_SYNC if sync is None else int(sync), _stream()),
           "attention_split")
    return out


def attention_oproj_tiles(n_out: int, target_wgs: int = 16) -> int:
    """16-column output tiles per workgroup for ``attention_oproj``: the divisor of N/16 in
    {2,3,4,5,6,8} whose workgroups-per-head count is closest to ``target_wgs``."""
    G = n_out // 16
    cands = [nt for nt in (2, 3, 4, 5, 6, 8) if G % nt == 0]
    if not cands:
        raise ValueError(f"attention_oproj: N/16 = {G} has no tile count in (2,3,4,5,6,8)")
    return min(cands, key=lambda nt: (abs(G // nt - target_wgs), nt))


def attention_oproj(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, row_slot: torch.Tensor,
                    row_kvlen: torch.Tensor, wo_sh: torch.Tensor, parts: torch.Tensor, scale: float | None = None,
                    tiles: int | None = None) -> torch.Tensor:
    """Decode attention fused with the out-projection (M <= 4 rows): head h's share
    ``attn_h(q) @ W_o[:, 64h:64h+64]^T`` goes to ``parts[h, :M, :N]`` (fp32 split-K slabs; no bias),
    so ``parts[:H].sum(0)`` is the out-projection -- what the next fused add+LN kernel sums with
    ``nsplit=H``.  ``wo_sh`` is ``shuffle_weight(W_o)`` with W_o [N, H*64]."""
    _req(q, torch.bfloat16, "q", 2)
    _req(k_cache, torch.bfloat16, "k_cache", 4)
    _req(v_cache, torch.bfloat16, "v_cache", 4)
    _req(row_slot, torch.int32, "row_slot", 1)
    _req(row_kvlen, torch.int32, "row_kvlen", 1)
    _req(wo_sh, torch.bfloat16, "wo_sh", 4)
    _req(parts, torch.float32, "parts", 3)
    M = q.shape[0]
    S, H, T, hd = k_cache.shape
    N = wo_sh.shape[0] * 16
    if not 1 <= M <= 4:
        raise ValueError("attention_oproj: 1..4 rows")
    if hd != 64 or v_cache.shape != k_cache.shape or q.shape[1] < H * 64 or wo_sh.shape[1] * 32 != H * 64:
        raise ValueError("attention_oproj: bad shapes")
    if parts.shape[0] < H or parts.shape[1] < M or parts.shape[2] < N or parts.stride(2) != 1:
        raise ValueError("attention_oproj: parts must be [>= H, >= M, >= N]")
    if row_slot.numel() < M or row_kvlen.numel() < M:
        raise ValueError("attention_oproj: index arrays too short")
    nt = attention_oproj_tiles(N) if tiles is None else tiles
    sc = (1.0 / 8.0) if scale is None else scale
    _check(lib().dlms_attention_oproj(_p(q), q.stride(0), _p(k_cache), _p(v_cache), _p(row_slot), _p(row_kvlen), M,
                                      H, T, S, float(sc), _p(wo_sh), N, int(nt), _p(parts), parts.stride(1),
                                      parts.stride(0), _stream()),
           "attention_oproj")
    return parts


def attention_oproj_grouped(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, row_slot: torch.Tensor,
                            row_kvlen: torch.Tensor, wo_sh: torch.Tensor, parts: torch.Tensor, heads_per_group: int,
                            scale: float | None = None, tiles: int = 3) -> torch.Tensor:
    """``attention_oproj`` for ONE row with heads in groups of ``heads_per_group`` (3 or 4): group g's
    share of the out-projection goes to ``parts[g, 0, :N]`` -- H / heads_per_group slabs."""
    _req(q, torch.bfloat16, "q", 2)
    _req(k_cache, torch.bfloat16, "k_cache", 4)
    _req(v_cache, torch.bfloat16, "v_cache", 4)
    _req(row_slot, torch.int32, "row_slot", 1)
    _req(row_kvlen, torch.int32, "row_kvlen", 1)
    _req(wo_sh, torch.bfloat16, "wo_sh", 4)
    _req(parts, torch.float32, "parts", 3)
    S, H, T, hd = k_cache.shape
    N = wo_sh.shape[0] * 16
    hg = int(heads_per_group)
    if q.shape[0] != 1:
        raise ValueError("attention_oproj_grouped: one row")
    if hd != 64 or v_cache.shape != k_cache.shape or q.shape[1] < H * 64 or wo_sh.shape[1] * 32 != H * 64:
        raise ValueError("attention_oproj_grouped: bad shapes")
    if hg not in (3, 4) or H % hg or (N // 16) % tiles or tiles not in (1, 2, 3, 4):
        raise ValueError("attention_oproj_grouped: heads_per_group in {3, 4} dividing H, tiles in 1..4 dividing N/16")
    if parts.shape[0] < H // hg or parts.shape[2] < N or parts.stride(2) != 1:
        raise ValueError("attention_oproj_grouped: parts must be [>= H/hg, >= 1, >= N]")
    sc = (1.0 / 8.0) if scale is None else scale
    _check(lib().dlms_attention_oproj_grouped(_p(q), _p(k_cache), _p(v_cache), _p(row_slot), _p(row_kvlen), H, hg, T,
                                              S, float(sc), _p(wo_sh), N, int(tiles), _p(parts), parts.stride(0),
                                              _stream()),
           "attention_oproj_grouped")
    return parts


# ---------------------------------------------------------------------------------------------
# Throughput-path decode GEMM: LDS-resident activation panel, pre-shuffled weights -> VGPRs
# ---------------------------------------------------------------------------------------------
PS_WAVES = 8


PS_LDS_BYTES = 160 * 1024  # gemm_ps.hip: activation panel (16 mt rows of kc * 2 + 32 B) + 8 x 4 KiB staging


def gemm_ps_geometry(M: int, N: int, epi: int, split: int = 1, cus: int = 256, K: int = 768):
    """(mt, nt, col_wgs) for ``gemm_ps``: 64-row blocks when the LM head's weight reuse matters
    and the K / split panel fits in LDS (K <= 1008: GPT-2-small; the wider models take 32-row
    blocks), else 32; column workgroups sized so the grid covers the CUs about once (the LM head
    loops over its tiles inside each wave)."""
    kc = K // max(1, split)
    fits4 = 64 * (kc * 2 + 32) + 8 * 4096 <= PS_LDS_BYTES
    mt = 4 if ((epi == EPI_ARGMAX or M >= 512) and fits4) else 2
    # (80-row LM-head panels, 7 passes over the 77 MB weight at 512 rows instead of 8, measured 1 %
    # slower at 1024 queries: profiles/r3_sweep_lmhead_mt.jsonl)
    nt = 2
    row_blocks = -(-M // (16 * mt))
    tiles = N // (16 * nt)
    need = -(-tiles // PS_WAVES)  # column workgroups for one tile per wave
    per_row = max(1, cus // max(1, row_blocks * split))
    col_wgs = min(need, per_row) if epi == EPI_ARGMAX else need
    return mt, nt, max(1, col_wgs)


def gemm_ps(a: torch.Tensor, w_sh: torch.Tensor, epi: int, *, bias=None, out=None, q_out=None, k_cache=None,
            v_cache=None, row_slot=None, row_pos=None, argmax_out=None, seen=None, vocab: int = 0,
            col_offset: int = 0, penalty: float = 1.0, split_k: int = 1, geometry=None):
    """C = a @ W.T for a ``shuffle_weight`` weight with the activation panel resident in LDS
    (``gemm_ps.hip``).  Same epilogue contract as ``gemm`` except EPI_ARGMAX: one key per
    (row, wave slot) -> ``argmax_out`` needs >= 8 * col_wgs columns (``gemm_ps_key_slots``)."""
    _req(a, torch.bfloat16, "a", 2)
    _req(w_sh, torch.bfloat16, "w_sh", 4)
    if w_sh.shape[2] != 64 or w_sh.shape[3] != 8 or not w_sh.is_contiguous():
        raise ValueError("gemm_ps: w_sh must be a contiguous shuffle_weight() tensor")
    N, K = w_sh.shape[0] * 16, w_sh.shape[1] * 32
    M = a.shape[0]
    if a.shape[1] != K or a.stride(0) % 8 or a.data_ptr() % 16:
        raise ValueError(f"gemm_ps: a {tuple(a.shape)} vs K={K} (16-byte aligned rows)")
    if split_k < 1 or K % split_k or (K // split_k) % 128:
        raise ValueError("gemm_ps: K / split_k must be a multiple of 128")
    if epi != EPI_PARTIAL and split_k != 1:
        raise ValueError("gemm_ps: split_k only with EPI_PARTIAL")
    mt, nt, col_wgs = geometry or gemm_ps_geometry(M, N, epi, split_k, K=K)
    if N % (16 * nt):
        raise ValueError("gemm_ps: N must be a multiple of 16 * nt")
    ep = GemmEpi()
    if bias is not None:
        _req(bias, torch.float32, "bias", 1)
        if bias.numel() < N:
            raise ValueError("bias too short")
        ep.bias = bias.data_ptr()
    if epi in (EPI_BF16, EPI_GELU_TANH):
        if out is None:
            out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
        _req(out, torch.bfloat16, "out", 2)
        if out.shape[0] < M or out.shape[1] < N or out.stride(0) % 8 or out.data_ptr() % 16:
            raise ValueError("gemm_ps: out too small / misaligned")
        ep.out, ep.ldo = out.data_ptr(), out.stride(0)
    elif epi == EPI_PARTIAL:
        if out is None:
            out = torch.empty(split_k, M, N, dtype=torch.float32, device=a.device)
        _req(out, torch.float32, "out", 3)
        if out.shape[0] < split_k or out.shape[1] < M or out.shape[2] < N or out.stride(1) % 4 or \
                out.stride(0) % 4 or out.data_ptr() % 16:
            raise ValueError("gemm_ps: partial out too small / misaligned")
        ep.out, ep.ldo, ep.split_k, ep.split_stride = out.data_ptr(), out.stride(1), split_k, out.stride(0)
    elif epi == EPI_QKV:
        for t, n in ((q_out, "q_out"), (k_cache, "k_cache"), (v_cache, "v_cache")):
            _req(t, torch.bfloat16, n)
        _req(row_slot, torch.int32, "row_slot", 1)
        _req(row_pos, torch.int32, "row_pos", 1)
        if N % 3 or (N // 3) % 64:
            raise ValueError("QKV N must be 3 * d_local (64-wide heads)")
        d_local = N // 3
        if k_cache.dim() != 4 or k_cache.shape != v_cache.shape or k_cache.shape[1] * 64 != d_local or \
                k_cache.shape[3] != 64 or not k_cache.is_contiguous() or not v_cache.is_contiguous():
            raise ValueError(f"cache shape {tuple(k_cache.shape)} incompatible with d_local={d_local}")
        if q_out.shape[0] < M or q_out.shape[1] < d_local or row_slot.numel() < M or row_pos.numel() < M or \
                q_out.stride(0) % 8 or q_out.data_ptr() % 16:
            raise ValueError("qkv epilogue buffers too small / misaligned")
        ep.q_out, ep.ldq = q_out.data_ptr(), q_out.stride(0)
        ep.k_cache, ep.v_cache = k_cache.data_ptr(), v_cache.data_ptr()
        ep.row_slot, ep.row_pos = row_slot.data_ptr(), row_pos.data_ptr()
        ep.n_heads, ep.t_max, ep.d_local, ep.n_slots = k_cache.shape[1], k_cache.shape[2], d_local, k_cache.shape[0]
        out = q_out
    elif epi == EPI_ARGMAX:
        _req(argmax_out, torch.int64, "argmax_out", 2)
        _req(seen, torch.int32, "seen", 2)
        slots = PS_WAVES * col_wgs
        if argmax_out.shape[0] < M or argmax_out.shape[1] < slots or seen.shape[0] < M or \
                seen.shape[1] * 32 < vocab or col_offset % 64:
            raise ValueError("gemm_ps argmax buffers too small / misaligned shard")
        ep.argmax_out, ep.ldo, ep.seen = argmax_out.data_ptr(), argmax_out.stride(0), seen.data_ptr()
        ep.seen_words, ep.vocab, ep.col_offset, ep.penalty = seen.stride(0), vocab, col_offset, penalty
        out = argmax_out
    else:
        raise ValueError(f"gemm_ps: unsupported epilogue {epi}")
    _check(lib().dlms_gemm_ps(epi, _p(a), a.stride(0), _p(w_sh), M, N, K, split_k, mt, nt, col_wgs, ctypes.byref(ep),
                              _stream()), "dlms_gemm_ps")
    return out


def gemm_ps_key_slots(M: int, N: int, K: int = 768) -> int:
    """argmax_out columns ``gemm_ps(..., EPI_ARGMAX)`` writes for an M x N x K LM head."""
    return PS_WAVES * gemm_ps_geometry(M, N, EPI_ARGMAX, K=K)[2]
