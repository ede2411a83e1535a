"""Build + load the hand-written gfx950 HIP kernel library (``libpto_hip.so``).

The kernels live in ``csrc/kernels/*.hip`` and are compiled in-tree with
``hipcc --offload-arch=gfx950`` into ``pytorch_operator_amd/_lib/libpto_hip.so``
(so the built object travels with a ``gpurun`` snapshot and is the one the
driver sees loaded).  The library exports a plain C ABI and is bound with
``ctypes``; every launcher validates shapes on the host before launching.

The library is linked against the HIP runtime by soname (``libamdhip64.so.7``);
``torch`` is always imported first so the process shares torch's already-loaded
HIP runtime (one runtime -> stream handles from ``torch.cuda`` are valid here).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import shutil
import subprocess
import tempfile
import threading
from pathlib import Path

import torch  # noqa: F401  (must be loaded before the HIP library, see module doc)

_PKG = Path(__file__).resolve().parent.parent
_ROOT = _PKG.parent
_SRC_DIR = _ROOT / "csrc" / "kernels"
_LIB_DIR = _PKG / "_lib"
_LIB_PATH = _LIB_DIR / "libpto_hip.so"
_STAMP = _LIB_DIR / "libpto_hip.stamp"
_ARCH = os.environ.get("PTO_OFFLOAD_ARCH", "gfx950")

_lock = threading.Lock()
_lib = None


class NativeLibraryError(RuntimeError):
    """Raised when the HIP kernel library cannot be built or loaded."""


def _sources():
    return sorted(_SRC_DIR.glob("*.hip")) + sorted(_SRC_DIR.glob("*.h"))


# Per-file compiler flags.  attention.hip: MFMAs in VGPR form -- its one-wave-per-SIMD dK/dV
# kernels need more than the 256 architectural VGPRs, and with the default (AGPR-form)
# accumulators the compiler moved them between AGPRs and VGPRs every tile (298 v_accvgpr_read +
# 261 v_accvgpr_write in the kernel against 31 + 22 with VGPR form).
# attention_bwd_pipe.hip: VGPR form as well (its dK/dV accumulators are pinned in AGPRs by its
# own asm MFMAs, so the compiler's MFMAs (S, dP) write VGPRs that the VALU reads directly), and
# no SLP vectorisation: packed f32 VALU beside MFMAs costs more issue time than two scalar ops
# (MI355X_MICROARCH.md, constants table).
_FILE_FLAGS = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
               "attention_bwd_pipe.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"]}


def _source_digest() -> str:
    h = hashlib.sha256()
    h.update(_ARCH.encode())
    h.update(repr(sorted(_FILE_FLAGS.items())).encode())
    for p in _sources():
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def hipcc_path() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise NativeLibraryError("hipcc not found (need ROCm: /opt/rocm/bin/hipcc)")


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile every ``csrc/kernels/*.hip`` for gfx950 into one shared library.

    Rebuilds only when the sources (or the target arch) changed.
    """
    digest = _source_digest()
    if not force and _LIB_PATH.exists() and _STAMP.exists() and _STAMP.read_text() == digest:
        return _LIB_PATH
    _LIB_DIR.mkdir(parents=True, exist_ok=True)
    hip_srcs = sorted(_SRC_DIR.glob("*.hip"))
    tmp = _LIB_PATH.with_suffix(f".so.tmp{os.getpid()}")
    objdir = Path(tempfile.mkdtemp(prefix="pto_hip_obj_"))
    base = [hipcc_path(), f"--offload-arch={_ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
            "-I", str(_SRC_DIR)]
    try:
        # one object per source (their own flags), compiled in parallel, then one shared library
        procs, objs = [], []
        for src in hip_srcs:
            obj = objdir / (src.stem + ".o")
            cmd = base + _FILE_FLAGS.get(src.name, []) + ["-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
            objs.append(str(obj))
        errs = []
        for src, pr in procs:
            _, err = pr.communicate()
            if pr.returncode != 0:
                errs.append(f"{src.name}: hipcc failed ({pr.returncode}):\n{err[-8000:]}")
        if errs:
            raise NativeLibraryError("\n".join(errs))
        cmd = [hipcc_path(), f"--offload-arch={_ARCH}", "-shared", "-fPIC", "-o", str(tmp), *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise NativeLibraryError(f"hipcc link failed ({res.returncode}):\n{res.stderr[-8000:]}")
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    os.replace(tmp, _LIB_PATH)
    _STAMP.write_text(digest)
    return _LIB_PATH


_VP = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_L = ctypes.c_long

_SIGNATURES = {
    "pto_mnist_conv1_fwd": [_VP, _I, _VP, _VP, _VP, _I, _I, _F, _F, _VP, _VP, _VP, _VP, _I, _VP,
                            _I, _VP, _VP, _VP],
    "pto_mnist_conv2_fwd": [_VP, _VP, _VP, _VP, _VP, _I, _VP],
    "pto_mnist_conv12_fwd": [_VP, _I, _VP, _VP, _VP, _I, _I, _F, _F] + [_VP] * 10 + [_I, _VP, _VP, _VP, _VP],
    "pto_slab_reduce_sgd": [_VP, _I, _I, _I, _VP, _VP, _VP, _F, _F, _F, _F, _F, _I, _I, _VP,
                            _VP, _VP, _VP, _I, _I, _I, _I, _VP],
    "pto_mnist_fc1_fwd": [_VP, _VP, _VP, _VP, _I, _VP],
    "pto_mnist_head": [_VP, _VP, _VP, _VP, _I, _F, _F, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP],
    "pto_mnist_fc1_fwd_parts": [_VP, _VP, _VP, _VP, _I, _VP],
    "pto_mnist_fc1_ks": [],
    "pto_mnist_fc1_bwd": [_VP] * 13 + [_F, _I, _I, _VP, _VP],
    "pto_mnist_conv_bwd": [_VP] * 10 + [_I, _I, _VP],
    "pto_slab_reduce": [_VP, _I, _I, _I, _VP, _I, _I, _I, _VP],
    "pto_mnist_synth": [_VP, _VP, _VP, _I, ctypes.c_uint, _F, _VP],
    "pto_mnist_conv_bwd4": [_VP] * 7 + [_I] * 6 + [_VP],
    "pto_mnist_fc1_bwd_stage": [_VP] * 13 + [_F, _I] + [_VP] * 4 + [_I, _I, _I, _VP, _VP, _VP, _VP, _VP],
    "pto_mnist_tail": [_VP, _I, _I, _I, _VP, _VP, _VP, _F, _F, _F, _F, _F, _I, _I, _VP, _I, _I, _I]
                      + [_VP] * 9 + [_F] + [_VP] * 7,
    "pto_mnist_tail_grads": [_VP, _I, _I, _I, _VP, _I, _I, _I] + [_VP] * 7 + [_F, _VP, _VP, _VP],
    "pto_mnist_fc1_bwd_head": [_VP] * 13 + [_F, _I] + [_VP] * 4 + [_I, _I, _VP, _VP, _VP, _VP, _VP],
    "pto_slab_reduce_sgd_w1": [_VP, _I, _I, _I, _VP, _VP, _VP, _F, _F, _F, _F, _F, _I, _I, _VP,
                               _VP, _VP, _VP, _I, _I, _I, _I] + [_VP] * 6,
    "pto_mnist_fc1_bwd_push": [_VP] * 13 + [_F, _I, _VP, _I, _I, _L, _L, _VP, _VP, _VP],
    "pto_sgd_momentum": [_VP, _VP, _VP, _L, _F, _F, _F, _F, _F, _I, _I, _VP, _VP],
    # xgmi_allreduce.hip
    "pto_xar_create": [_I, _I, _L, _I, ctypes.c_double, ctypes.POINTER(_VP), _VP],
    "pto_xar_open": [_VP, _VP],
    "pto_xar_error": [_VP],
    "pto_xar_stamps": [_VP, _VP, _I],
    "pto_xar_prebarrier": [_VP, _I],
    "pto_xar_reset": [_VP],
    "pto_xar_fence": [_VP, _I],
    "pto_xar_resident_blocks": [_VP, _I],
    "pto_xar_alloc_kind": [_VP],
    "pto_xar_allreduce": [_VP, _VP, _VP, _F, _VP],
    "pto_xar_allreduce_sgd": [_VP, _VP, _VP, _VP, _F, _F, _F, _F, _F, _I, _I, _VP, _VP, _I, _L, _L,
                              _I, _L, _L, _L, _L, _VP],
    "pto_xar_allreduce_sgd_fc": [_VP, _VP, _VP, _VP, _F, _F, _F, _F, _F, _I, _I, _VP, _VP, _I, _L, _L,
                                 _I, _L, _L] + [_VP] * 6 + [_F, _I, _L, _L, _L, _L, _VP],
    "pto_xar_push_info": [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_L)],
    "pto_xar_destroy": [_VP],
    "pto_xar_emu_create": [_I, _L, _I, ctypes.c_double, _I, _I, ctypes.POINTER(_VP)],
    "pto_xar_emu_set": [_VP, _I, _VP, _VP, _VP, _VP, _I, _L, _L, _I, _L, _L, _F, _F, _F, _F, _I, _I, _L, _L],
    "pto_xar_emu_set_fc": [_VP] + [_VP] * 6 + [_I, _F, _L, _L, _L, _L],
    "pto_xar_emu_prepush": [_VP, _VP],
    "pto_xar_emu_launch": [_VP, _VP],
    "pto_xar_emu_error": [_VP],
    "pto_xar_emu_threads": [_VP],
    "pto_xar_emu_destroy": [_VP],
    # rmsnorm.hip
    "pto_rmsnorm_fwd": [_VP, _VP, _VP, _VP, _L, _I, _F, _I, _VP],
    "pto_rmsnorm_bwd": [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _L, _I, _I, _I, _VP],
    "pto_add_rmsnorm_fwd": [_VP, _VP, _VP, _VP, _VP, _VP, _L, _I, _F, _I, _VP],
    "pto_add_rmsnorm_bwd": [_VP] * 9 + [_L, _I, _I, _I, _VP],
    # llm_fused.hip
    "pto_rope": [_VP, _VP, _VP, _VP, _L, _I, _I, _I, _F, _I, _VP],
    "pto_swiglu_fwd": [_VP, _VP, _VP, _L, _I, _VP],
    "pto_swiglu_bwd": [_VP, _VP, _VP, _VP, _VP, _L, _I, _VP],
    "pto_rope_qkv": [_VP] * 6 + [_L, _I, _I, _I, _I, _I, _I, _VP],
    "pto_swiglu_packed_fwd": [_VP, _VP, _L, _I, _I, _VP],
    "pto_swiglu_packed_bwd": [_VP, _VP, _VP, _L, _I, _I, _VP],
    "pto_transpose16": [_VP, _VP, _L, _L, _VP],
    "pto_xent_fwd": [_VP, _VP, _VP, _VP, _L, _I, _L, _I, _VP],
    "pto_xent_bwd": [_VP, _VP, _VP, _VP, _VP, _L, _I, _L, _I, _VP],
    # adamw.hip
    "pto_adamw_step": [_VP, _VP, _VP, _VP, _VP, _L, _I, _F, _F, _F, _F, _F, _I, _VP],
    "pto_adamw_step_scaled": [_VP, _VP, _VP, _VP, _VP, _L, _I, _F, _F, _F, _F, _F, _I, _F, _VP],
    # batchnorm.hip
    "pto_bn_plan": [_L, _I, ctypes.POINTER(_I)],
    "pto_bn_fwd_train": [_VP] * 12 + [_L, _I, _I, _I, _F, _F, _I, _I, _VP, _VP],
    "pto_bn_bwd": [_VP] * 14 + [_L, _I, _I, _I, _I, _I, _VP],
    # attention.hip
    "pto_attn_fwd": [_VP] * 5 + [_I] * 5 + [_F, _I, _VP],
    "pto_attn_bwd": [_VP] * 10 + [_I] * 5 + [_F, _I, _VP],
    "pto_attn_set_variant": [_I],
    "pto_attn_set_dkdv_variant": [_I],
    "pto_attn_set_dq_variant": [_I],
    # pool.hip
    "pto_maxpool3s2_fwd": [_VP, _VP, _VP, _I, _I, _I, _I, _VP],
    "pto_maxpool3s2_bwd": [_VP, _VP, _VP, _I, _I, _I, _I, _VP],
    # graph_exec.hip
    "pto_graph_begin": [_VP],
    "pto_graph_end": [_VP, ctypes.POINTER(_VP)],
    "pto_graph_upload": [_VP, _VP],
    "pto_graph_launch": [_VP, _VP, _I],
    "pto_graph_launch_stream": [_VP, _VP, _I],
    "pto_graph_launch_stream_probe": [_VP, _VP, _VP, _I, _I, _I, _I],
    "pto_graph_destroy": [_VP],
    "pto_device_prewarm": [_I, _VP, _VP],
}
_LONG_FNS = {"pto_xar_npad": [_VP], "pto_xar_emu_npad": [_VP], "pto_rmsnorm_bwd_parts": [_L, _I],
             "pto_graph_nodes": [_VP]}
_VOID_FNS = {"pto_set_debug_buffer": [_VP], "pto_xar_emu_stamps": [_VP, _VP]}
_PTR_FNS = {"pto_xar_err_ptr": [_VP]}


def load(build_if_missing: bool = True):
    """Return the loaded ``ctypes.CDLL`` (building it first if needed)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # PTO_HIP_LIB: load a prebuilt variant instead (kernel A/B experiments, tools/exp_*.sh)
        path = Path(os.environ["PTO_HIP_LIB"]) if os.environ.get("PTO_HIP_LIB") else _LIB_PATH
        if build_if_missing and path == _LIB_PATH:
            build()
        if not path.exists():
            raise NativeLibraryError(f"{path} missing; run pytorch_operator_amd.ops.build()")
        lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        variant = path != _LIB_PATH  # an A/B build may predate entry points it never exercises
        for table, restype in ((_SIGNATURES, ctypes.c_int), (_LONG_FNS, ctypes.c_long), (_VOID_FNS, None),
                               (_PTR_FNS, ctypes.c_void_p)):
            for name, argtypes in table.items():
                try:
                    fn = getattr(lib, name)
                except AttributeError:
                    if variant:
                        continue
                    raise
                fn.argtypes = argtypes
                fn.restype = restype
        _lib = lib
        return lib


def library_path() -> Path:
    return Path(os.environ["PTO_HIP_LIB"]) if os.environ.get("PTO_HIP_LIB") else _LIB_PATH


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def current_stream_ptr(device=None) -> int:
    """The current HIP stream of ``device`` (default: the current device) as an integer handle.
    Uses torch's raw-pointer accessor (no ``torch.cuda.Stream`` object per call: a few us less
    host time before every launch -- the first launch of a timed region included)."""
    if _raw_stream is not None:
        idx = torch.cuda.current_device() if device is None else (
            device.index if isinstance(device, torch.device) and device.index is not None else
            (torch.cuda.current_device() if isinstance(device, torch.device) else int(device)))
        return int(_raw_stream(idx))
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise NativeLibraryError(f"{what} failed with code {rc}")
