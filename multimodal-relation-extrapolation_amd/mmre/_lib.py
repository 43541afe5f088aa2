"""ctypes binding of libmmre_hip.so (the C ABI declared in include/mmre.h).

The library is the only compute path: if it is missing or cannot load, every op
raises -- there is no CPU or eager-PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first: libmmre_hip binds to the same libamdhip64.so.7)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.environ.get("MMRE_LIB") or os.path.join(LIB_DIR, "libmmre_hip.so")

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
F32 = ctypes.c_float

# name -> (restype, argtypes)
SIGNATURES = {
    "mmre_version": (I32, []),
    "mmre_link_k": (I64, [I32, I32]),
    "mmre_link_pad": (I64, [I64]),
    "mmre_link_prepare_entities": (I32, [I32, I32, P, P, I64, I32, P, I64, P, P]),
    "mmre_link_prepare_queries": (I32, [I32, I32, P, P, P, I64, I64, I32, F32, P, P, P, P, I64, P, I64, P, P, P, P]),
    "mmre_link_truth": (I32, [I32, I32, F32, P, I64, I64, P, P, P, P, P, I64, I64, I32, P, P, P, P, P, P, P]),
    "mmre_link_truth_grouped": (I32, [I32, I32, F32, P, I64, P, P, P, P, I64, I32, P, P, I64, P, P, P, I64, P, P, P,
                                      P, P, P]),
    "mmre_link_sweep": (I32, [I32, I32, F32, P, I64, I64, P, P, P, P, I64, I64, I32, P, P, P, P, P, P]),
    "mmre_link_sweep_range": (I32, [I32, I32, F32, P, I64, I64, I64, I64, P, P, P, P, I64, I64, I32, P, P, P, P, P]),
    "mmre_link_l1q_workspace": (I64, [I32, I64, I64]),
    "mmre_link_l1q_stats": (I32, [P, I64, P, P]),
    "mmre_link_sweep_l1q": (I32, [I32, F32, P, P, I64, I64, I64, I64, P, P, P, P, P, I64, I64, I32, P, P, P, P, P,
                                  I64, P]),
    "mmre_link_evaluate_l1q_workspace": (I64, [I32, I64, I64]),
    "mmre_link_evaluate_l1q": (I32, [I32, P, I64, P, I64, I32, P, P, P, P, I64, P, P, I64, P, P, P, I64, I64, I64, P,
                                     I64, P, P, I64, P, P, P, P, P, P, P, I64, P]),
    "mmre_link_bf3_workspace": (I64, [I32, I32, I64, I64]),
    "mmre_link_bf3_stats": (I32, [P, I64, P, P]),
    "mmre_link_sweep_bf3": (I32, [I32, I32, F32, P, P, I64, I64, I64, I64, P, P, P, P, P, I64, I64, I32, P, P, P,
                                  I64, P]),
    "mmre_link_sweep_bf3_rows": (I32, [I32, I32, F32, P, I64, I64, I64, I64, P, P, P, P, P, P, I64, I64, I32, P, P,
                                       P, I64, P]),
    "mmre_link_metrics": (I32, [P, P, I64, I64, P]),
    "mmre_glibc_rand": (I32, [I64, I64, P]),
    "mmre_sampler_advance": (I32, [P, I64, I64, I64, I64, I64]),
    "mmre_sampler_advance_device": (I32, [P, I64, I64, I64, I64, I64, P]),
    "mmre_sampler_draws_per_positive": (I64, [I64, I64, I64]),
    "mmre_sampler_openke": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P, I64, I64, P, I64, I64, I64, I64, I64,
                                  P, P, P, P, P]),
    "mmre_sampler_blocks": (I32, [P, I64, P, P, P, P, P, P, P, P]),
    "mmre_sampler_openke_blocked": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P, I64, I64, P, I64, I64, I64, I64,
                                          I64, P, I64, P, P, P, P, P]),
    "mmre_sampler_openke_step": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P, I64, I64, P, I64, I64, I64, I64,
                                       I64, P, I64, P, P, P, P, P, P]),
    "mmre_sampler_openke_p": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P, I64, I64, P, I64, I64, I64, I64,
                                    I64, P, I64, P, P, P, P, P, P, P]),
    "mmre_import_prob": (I32, [ctypes.c_char_p, I64, F32, P]),
    "mmre_sampler_repo": (I32, [P, P, P, I64, I64, I64, P, I64, P, P, P, I64, P, P, P, I64, ctypes.c_uint64, I32,
                                P, P, P, P]),
    "mmre_sgd_step": (I32, [P, P, P, I32, F32, P]),
    "mmre_ns_workspace": (I64, [I64, I64]),
    "mmre_ns_forward": (I32, [I32, I32, F32, I32, P, P, P, P, I32, F32, P, P, P, I64, I64, F32, F32, F32, P, P, P,
                              P]),
    "mmre_ns_backward": (I32, [I32, I32, F32, I32, P, P, P, P, I32, F32, P, P, P, I64, I64, F32, F32, F32, P, P, P,
                               P, P, P, I64, I64, P, I64, P]),
    "mmre_rows_backward_workspace": (I64, [I32, I64, I64, I64, I32]),
    "mmre_ns_fused_workspace": (I64, [I32, I32, I64, I64, I64, I64, I32]),
    "mmre_ns_fused_forward": (I32, [I32, I32, F32, I32, P, P, P, P, I64, I64, I32, F32, P, P, P, I64, I64, F32, F32,
                                    F32, P, P, P, P]),
    "mmre_ns_fused_grad": (I32, [I32, I32, F32, I32, P, P, P, P, I64, I64, I32, F32, P, P, P, I64, I64, F32, F32, F32,
                                 P, P, P, P, P, P, P, P]),
    "mmre_ns_fused_grad_sgd": (I32, [I32, I32, F32, I32, P, P, P, P, I64, I64, I32, F32, P, P, P, I64, I64, F32, F32,
                                     F32, P, P, P, P, P, P, P, F32, P]),
    "mmre_ns_step_openke": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P, P, I64, I64, P, I64, P, P, P, P, P, I32, I32,
                                  P, P, I64, I64, I32, I64, I64, F32, F32, F32, P, P, P, P, P, F32, P]),
    "mmre_ns_step_openke_gen_pipe": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P, P, I64, I64, P, I64, P, P, P, P, P,
                                           I32, F32, I32, P, P, P, P, I64, I64, I32, F32, I64, I64, F32, F32, F32, P,
                                           P, P, P, P, P, P, F32, P, I64, P, P, P, P]),
    "mmre_ns_step_openke_pipe": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P, P, I64, I64, P, I64, P, P, P, P, P, I32,
                                       I32, P, P, I64, I64, I32, I64, I64, F32, F32, F32, P, P, P, P, P, F32, P, I64,
                                       I64, P, P, P, P]),
    "mmre_ns_forward_backward": (I32, [I32, I32, F32, I32, P, P, P, P, I64, I64, I32, F32, P, P, P, I64, I64, F32, F32,
                                       F32, P, P, P, P, P, P, P, P]),
    "mmre_score_rows_backward": (I32, [I32, I32, F32, I32, P, P, P, P, I32, F32, P, P, P, I64, P, P, P, P, P, I64, I64,
                                       P, I64, P]),
    "mmre_generator_workspace": (I64, [I64, I32, I32, I32, I32]),
    "mmre_generator_forward": (I32, [P, I32, P, I32, I64, P, P, P, P, I32, P, P, P, P, I32, P, P, P, P, I32, P, P,
                                     F32, I32, F32, P, P, P]),
    "mmre_generator_forward_save": (I32, [P, I32, P, I32, I64, P, P, P, P, I32, P, P, P, P, I32, P, P, P, P, I32,
                                          P, P, F32, I32, F32, P, P, P, P]),
    "mmre_generator_acts_size": (I64, [I64, I32, I32, I32, I32]),
    "mmre_generator_backward_workspace": (I64, [I64, I32, I32, I32, I32]),
    "mmre_generator_backward": (I32, [P, I64, I32, I32, I32, I32] + [P] * 12 + [F32] + [P] * 10),
    "mmre_candidate_rank_transe": (I32, [P, P, I32, P, P, I64, P, P, P, P, P]),
    "mmre_cosine_rank": (I32, [P, I32, P, I64, P, I32, P, P, P, P]),
    "mmre_extractor_pack_size": (I64, [I32]),
    "mmre_extractor_pack": (I32, [I32] + [P] * 15 + [P]),
    "mmre_extractor_nodes": (I32, [I32, P, P, P, P, I32, P, I64, P, P, P]),
    "mmre_extractor_encode": (I32, [I32, P, F32, P, P, P, P, I64, P, P, I32, P, P, P]),
    "mmre_extractor_targets": (I32, [P, I64, I32, I32, I32, P, P]),
    "mmre_rank_desc": (I32, [P, P, I64, P, P]),
    "mmre_extractor_train_inputs": (I32, [I32, P, P, P, P, I32, I64, F32, P, P, P, P, P, P, P, P, P]),
    "mmre_dropout": (I32, [P, P, P, I64, F32, P, I32, P]),
    "mmre_m3ae_max_len": (I32, []),
    "mmre_m3ae_plan_size": (I64, [I64]),
    "mmre_m3ae_plan": (I32, [P, P, I64, I64, I32, I64, P, P]),
    "mmre_m3ae_workspace": (I64, [I64, I64, I32]),
    "mmre_m3ae_encode": (I32, [P, I32, I32, I32, F32, P, P, I64, I64, I64, P, I64, I64, I32, P, I64, P, P]),
    "mmre_m3ae_layernorm": (I32, [P, I64, I32, P, P, F32, P, P]),
    "mmre_m3ae_linear": (I32, [I32, P, I64, I32, P, I32, P, P, P, P]),
    "mmre_m3ae_attention": (I32, [P, P, I64, I32, I32, I32, F32, I32, P, P]),
    "mmre_gemm_splits": (I32, [I64, I64, I64]),
    "mmre_gemm_f32": (I32, [P, I64, I64, P, I64, I64, I64, I64, I64, P, P, P]),
    "mmre_sn_weight": (I32, [P, I32, I32, P, P, I32, F32, P, P, P, P, P, P]),
    "mmre_sn_weight_backward": (I32, [P, P, I32, I32, P, P, P, P, P]),
    "mmre_layernorm_unbiased": (I32, [P, I64, I32, P, P, F32, P, P]),
    "mmre_layernorm_unbiased_backward": (I32, [P, P, I64, I32, P, F32, P, P, P, P, P]),
}

ERRORS = {1: "bad argument", 2: "unknown model", 3: "unsupported shape", 4: "workspace too small"}

_lib = None


class MMREError(RuntimeError):
    pass


def lib():
    """Load libmmre_hip.so once; raise loudly when it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MMREError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                            f"(make -C multimodal-relation-extrapolation_amd). There is no fallback path.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue  # call() raises for a symbol this build does not export
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def lib_identity() -> dict:
    """Which binary the process runs: path, size and sha256 prefix of libmmre_hip.so (the bench
    records it, so a result names the exact build that produced it)."""
    import hashlib
    with open(LIB_PATH, "rb") as f:
        blob = f.read()
    return {"path": os.path.relpath(LIB_PATH, os.path.dirname(os.path.dirname(os.path.dirname(LIB_PATH)))),
            "bytes": len(blob), "sha256": hashlib.sha256(blob).hexdigest()[:16]}


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        if rc >= 1000:
            raise MMREError(f"{what}: HIP error {rc - 1000}")
        raise MMREError(f"{what}: {ERRORS.get(rc, 'error')} (code {rc})")


def call(name: str, *args):
    fn = getattr(lib(), name, None)
    if fn is None:
        raise MMREError(f"{LIB_PATH} does not export {name}: rebuild it")
    rc = fn(*args)
    check(rc, name)
    return rc


def ptr(t):
    """Device/host pointer of a tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def mark_written(*tensors):
    """Bump torch's version counter of tensors a C-ABI call rewrote in place through raw pointers
    (torch's own in-place ops do this; a raw-pointer writer must do it itself), so that version
    checks -- autograd's saved-tensor check, OpenKETrainStep's prefetch validity -- see the write."""
    from torch.autograd.graph import increment_version
    for t in tensors:
        if t is not None:
            increment_version(t)


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise MMREError("mmre ops take device tensors (the HIP path is the only path)")
