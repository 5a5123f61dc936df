"""Autograd wrappers over the libmdemi C ABI.

Every function here runs the hand-written gfx950 kernels through ``_lib``;
there is no eager/ATen fallback for the math (torch supplies device memory,
streams and the autograd tape).  Activations are channels-last: token-major
``[rows, C]`` tensors and NHWC feature maps.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib as L

# --------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------


def _require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("mdemi ops run on the GPU only; got a CPU tensor")
        if t is not None and t.dtype != torch.float32:
            raise ValueError(f"mdemi ops are fp32; got {t.dtype}")


def _c(t):
    return t if t is None or t.is_contiguous() else t.contiguous()


def _target_blocks():
    return _SPLIT_TARGET_BLOCKS


_SPLIT_TARGET_BLOCKS = int(os.environ.get("MDEMI_SPLIT_TARGET_BLOCKS", "1024"))


def _split_for(M, N, K):
    """Split-K factor so that a long reduction still fills the chip.  Skinny outputs (fewer
    than 8 tiles: the weight gradients of narrow 1x1 convs over ~10^6 pixels) split up to 512
    ways; their slabs are combined by a column sum."""
    tiles = math.ceil(M / 128) * math.ceil(N / 128)
    ktiles = math.ceil(K / 16)
    # tools/gemm_split_study.py (profiles/r02_split_study.log): >= 384 output tiles already
    # fill the chip (a split only adds slab traffic); each split keeps >= 512 rows of K, 256
    # under bf16, whose workgroups finish a k-tile several times faster (bf16 Depthformer
    # 78.95 -> 77.44 ms; fp32 NeW-CRFs unchanged, AdaBins within noise; 128 slower again --
    # tools/gpu_r4r.sh, gpu_r4s.sh, profiles/round4/ab_split_min_rows.txt)
    bf16 = get_matmul_precision() == "bf16"
    min_kt = _SPLIT_MIN_KTILES if bf16 else 32
    if ktiles < min_kt:
        return 1
    # fp32 only: narrower outputs keep the deep splits they need; bf16 workgroups finish a
    # k-tile several times faster, so there the slab combine dominates and the round-4 rule
    # measured better (Depthformer bf16 140.3 vs 138.2 img/s, profiles/round5/ab_split_policy.txt)
    if tiles >= 32 and not bf16 and _SPLIT_POLICY == "fill":
        if 384 <= tiles <= 512:  # one round at two workgroups per CU already: a split only adds slabs
            return 1            # (9600x768x3072: split 5 measured 112 vs 118 TF/s unsplit)
        return _split_fill(tiles, min(ktiles // min_kt, 128), 1 if tiles >= 384 else min(
            max(1, _target_blocks() // tiles), ktiles // min_kt, 128))
    if tiles >= 384:
        return 1
    target, cap = (_target_blocks(), 128) if tiles >= 8 else (2 * _target_blocks(), 512)
    split = min(max(1, target // tiles), ktiles // min_kt, cap)
    return max(1, split)


_SPLIT_POLICY = os.environ.get("MDEMI_SPLIT_POLICY", "fill")  # "legacy": the round-4 rule (A/B)


def _split_fill(tiles, smax, s_legacy):
    """Split factor by wave quantisation: the tiles x split workgroups run in rounds of one per
    CU, so a split whose last round is nearly empty wastes that round (768x768x9600: 36 tiles x
    18 = 648 workgroups = 2.5 rounds, 147 us; x 7 = 252 = one full round, 126 us).  Cost per
    unit of work: rounds / split, times 1 % per split for the slab traffic and the last
    arriver's serial combine (tools/gemm_split_study.py, profiles/round5/split_study.txt).  The
    round-4 rule's factor stays unless this one is >= 5 % cheaper by the model."""
    cus = _device_cus()

    def cost(s):
        return -(-tiles * s // cus) / s * (1.0 + 0.01 * s)

    best = min(range(1, max(1, smax) + 1), key=lambda s: (cost(s), s))
    return best if cost(best) < 0.95 * cost(s_legacy) else s_legacy


_SPLIT_MIN_KTILES = int(os.environ.get("MDEMI_SPLIT_MIN_KTILES", "16"))  # bf16; K tiles of 16 rows
_CUS = [int(os.environ.get("MDEMI_CUS", "0"))]  # > 0: override the compute-unit count (A/B runs)


def _device_cus():
    """Compute units of the current device (the split model's round size), read once."""
    if _CUS[0] <= 0:
        try:
            _CUS[0] = int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
        except (RuntimeError, AssertionError):
            _CUS[0] = 256  # MI355X; only reached without a GPU (the CPU tests of the split plan)
    return _CUS[0]


def _draw_seed(device):
    """A dropout seed drawn on the GPU (torch's Philox; graph-safe: a captured step draws a new
    one on every replay).  Kernels read it through mdemi_dropout_dev."""
    return torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)


# Attention dropout fused into the softmax sweep (the bf16 copy of dropout(P), reused for dV):
# the same mask and values as the standalone sweeps, bit for bit; MDEMI_FUSE_DROPOUT=0 keeps the
# sweeps (A/B).  (A dropout stage in the GEMM epilogue was measured and removed: DESIGN.md §5.)
_FUSE_DROP = [os.environ.get("MDEMI_FUSE_DROPOUT", "1") != "0"]


def _drop(src_ptr, dst_ptr, n, p, seed, add=0, offset=0, dst16_ptr=None):
    """Inverted dropout of n floats; mask = hash(seed[0] + add, offset + i); dst16_ptr: also
    the bf16 copy of the result."""
    L.call("mdemi_dropout_dev16", src_ptr, dst_ptr, dst16_ptr, n, float(p), seed.data_ptr(), add, offset,
           L.stream())


# Matmul precision of every libmdemi GEMM:
#   "fp32"  exact-product fp32 MFMA (v_mfma_f32_32x32x2_f32), the reference's precision;
#   "fp32e" fp32 on the bf16 matrix cores: operands split exactly into three bf16 planes,
#           six plane products, fp32 accumulation at 2.67x the fp32 peak
#           (mdemi_gemm_f32e); fp32-level error except on heavily cancelling sums
#           (DESIGN.md §5), hence opt-in;
#   "bf16"  bf16 operands, fp32 accumulate: torch.autocast's matmul numerics (BASELINE
#           configs[4]).
# Process-wide; set it for a whole train step (forward and backward).
PRECISIONS = ("fp32", "fp32e", "bf16")
_PRECISION = [os.environ.get("MDEMI_MATMUL_PRECISION", "fp32")]
if _PRECISION[0] not in PRECISIONS:
    raise ValueError(f"MDEMI_MATMUL_PRECISION must be one of {PRECISIONS}, got {_PRECISION[0]!r}")


def set_matmul_precision(precision: str) -> None:
    if precision not in PRECISIONS:
        raise ValueError(f"matmul precision must be one of {PRECISIONS}, got {precision!r}")
    _PRECISION[0] = precision


def get_matmul_precision() -> str:
    return _PRECISION[0]


# bf16 storage of GEMM operands (precision "bf16"): every GEMM whose operands the DMA loaders
# can stage reads bf16 copies (mdemi_gemm_bf16x) -- written by the producing kernel where it
# can (set_b16), else by one cast sweep on first use, reused by every later GEMM on the same
# tensor (the forward product and the weight gradient read the same activation).  The copies
# are the RNE bf16 the fp32-operand bf16 GEMM rounds to as it stages, so results are
# bit-identical; only bias-gradient row sums move from the GEMM to a column-sum sweep over the
# same fp32 values.  MDEMI_BF16_STORAGE=0 (or set_bf16_storage(False)) keeps every operand fp32.
_B16_STORAGE = [os.environ.get("MDEMI_BF16_STORAGE", "1") != "0"]


def set_bf16_storage(on: bool) -> None:
    _B16_STORAGE[0] = bool(on)


def get_bf16_storage() -> bool:
    return _B16_STORAGE[0]


# Parameters change in place through raw pointers (FusedAdamW's kernel), which torch's version
# counter does not see: their bf16 copies are valid for one weight epoch, bumped by every
# optimizer step (bump_weight_epoch), so each weight is cast once per train step and its copy
# shared by the forward product and the data gradient.
_W_EPOCH = [0]


def bump_weight_epoch() -> None:
    _W_EPOCH[0] += 1


def set_b16(t, b16):
    """Record b16 (a bf16 tensor, t's shape, contiguous) as the RNE bf16 copy of t; valid
    while t is not modified in place (t._version; parameters: for this weight epoch)."""
    t._mdemi_b16 = (b16, t._version, _W_EPOCH[0])
    return t


def _b16_rec(t, numel):
    rec = t.__dict__.get("_mdemi_b16")
    if rec is None or rec[1] != t._version or rec[0].numel() != numel:
        return None
    if t.is_leaf and t.requires_grad and rec[2] != _W_EPOCH[0]:
        return None
    return rec[0]


_B16_CHECK = os.environ.get("MDEMI_B16_CHECK") == "1"


def _b16_checked(t, b):
    """MDEMI_B16_CHECK=1: every reuse of a recorded bf16 copy is compared with a fresh RNE cast
    of the fp32 tensor (a raw in-place write that torch's version counter did not see would
    otherwise hand a stale operand to a bf16 GEMM silently)."""
    if not _B16_CHECK:
        return b
    fresh = torch.empty(t.shape, dtype=torch.bfloat16, device=t.device)
    L.call("mdemi_cast_bf16", t.data_ptr(), fresh.data_ptr(), t.numel(), L.stream())
    if not torch.equal(fresh.view(torch.int16), b.view(t.shape).view(torch.int16)):
        raise RuntimeError(f"stale bf16 copy of a {tuple(t.shape)} tensor (MDEMI_B16_CHECK)")
    return b


def b16_of(t, convert=True):
    """The bf16 copy of contiguous fp32 tensor t: the recorded one (set_b16; on t or on the
    tensor t is a whole view of) if still valid, else (convert) a cast sweep, recorded on t --
    or on the parameter t views.  None for a tensor that cannot be copied this way
    (non-contiguous, unaligned)."""
    b = _b16_rec(t, t.numel())
    if b is not None:
        return _b16_checked(t, b)
    base = t._base
    whole = base is not None and base.data_ptr() == t.data_ptr() and base.numel() == t.numel()
    if whole:
        b = _b16_rec(base, t.numel())
        if b is not None:
            return _b16_checked(t, b.view(t.shape))
    if not convert or not t.is_contiguous() or t.data_ptr() % 16 or t.dtype != torch.float32:
        return None
    b = torch.empty(t.shape, dtype=torch.bfloat16, device=t.device)
    L.call("mdemi_cast_bf16", t.data_ptr(), b.data_ptr(), t.numel(), L.stream())
    set_b16(base if (whole and base.is_contiguous()) else t, b if not (whole and base.is_contiguous())
            else b.view(base.shape))
    return b


def new_b16_like(t):
    """A bf16 buffer for a producer to write t's copy into (bf16 storage on), else None."""
    if _PRECISION[0] != "bf16" or not _B16_STORAGE[0]:
        return None
    return torch.empty(t.shape, dtype=torch.bfloat16, device=t.device)


# autograd nodes whose backward runs bf16 GEMMs on the gradient of their output
_GEMM_BWD_NODES = frozenset(("_LinearFnBackward", "_Conv2dFnBackward", "_Conv2dSkipFnBackward", "_MlpFnBackward",
                             "_LinearActFnBackward", "_AttentionFnBackward", "_BatchedGemmFnBackward"))


def grad_feeds_gemm(x):
    """True (bf16 storage on) when x came from an op whose backward reads x's gradient as a
    bf16 GEMM operand: the op producing that gradient then writes its bf16 copy too."""
    return (_PRECISION[0] == "bf16" and _B16_STORAGE[0] and x.grad_fn is not None
            and type(x.grad_fn).__name__ in _GEMM_BWD_NODES)


class matmul_precision:
    """Context manager: with matmul_precision("bf16"): ..."""

    def __init__(self, precision):
        self.precision, self.prev = precision, None

    def __enter__(self):
        self.prev = get_matmul_precision()
        set_matmul_precision(self.precision)
        return self

    def __exit__(self, *a):
        set_matmul_precision(self.prev)
        return False


# the path the last gemm() call took ("b16": bf16 operands in HBM; else the precision) -- for
# the benchmark's per-family roofline, which prices bf16 operands at 2 bytes
LAST_GEMM = ["fp32"]


def gemm(A, B, C, M, N, K, *, lda, ldb, ldc, a_layout, b_layout, a_op=L.OP_NONE, b_op=L.OP_NONE,
         alpha=1.0, beta=0.0, bias=None, bias_mode=L.BIAS_NONE, act=L.ACT_NONE, aux=None, ldaux=0,
         residual=None, ldres=0, batch=1, a_bstride=0, b_bstride=0, c_bstride=0, aux_bstride=0,
         res_bstride=0, split_k=None, conv=None, preact=None, ldpre=0, pre_bstride=0, rowsum_a=None,
         a_off=0, b_off=0, c_off=0, inner=None, row_scale=None, row_scale_group=0, a16=None, b16=None, c16=None):
    """a_off/b_off/c_off: element offsets into A/B/C (column slices of wider buffers).
    inner=(n, a_bstride_inner, b_bstride_inner, c_bstride_inner): a two-level batch of
    batch = outer * n entries (mdemi_gemm_desc.batch_inner), e.g. (image, head).
    a16 / b16 / c16 (precision "bf16" only): bf16 copies of A / B (the RNE bf16 of the fp32
    tensors, same layout; A / B may then be None) and a bf16 copy of C to write -- the bf16
    storage path (mdemi_gemm_bf16x), bit-identical to the fp32-operand bf16 GEMM.  With A (or
    B) None only the bf16 copy exists: B16Unsupported is raised (before any launch) when the
    bf16 loaders cannot stage this layout."""
    if inner is not None and inner[0] > 1 and os.environ.get("MDEMI_GEMM_SPLIT_INNER") == "1":
        # debug/A-B path: the same products as one launch per inner index
        n, a2, b2, c2 = inner
        for i in range(n):
            gemm(A, B, C, M, N, K, lda=lda, ldb=ldb, ldc=ldc, a_layout=a_layout, b_layout=b_layout, a_op=a_op,
                 b_op=b_op, alpha=alpha, beta=beta, bias=bias, bias_mode=bias_mode, act=act, batch=batch // n,
                 a_bstride=a_bstride, b_bstride=b_bstride, c_bstride=c_bstride, split_k=split_k, conv=conv,
                 a_off=a_off + i * a2, b_off=b_off + i * b2, c_off=c_off + i * c2)
        return C
    d = L.GemmDesc()
    d.M, d.N, d.K, d.batch = M, N, K, batch
    if inner is not None and inner[0] > 1:
        d.batch_inner, d.a_bstride_inner, d.b_bstride_inner, d.c_bstride_inner = inner
    d.A = A.data_ptr() + 4 * a_off if A is not None else None
    d.B = B.data_ptr() + 4 * b_off if B is not None else None
    d.lda, d.a_bstride, d.a_layout, d.a_op = lda, a_bstride, a_layout, a_op
    d.ldb, d.b_bstride, d.b_layout, d.b_op = ldb, b_bstride, b_layout, b_op
    d.C, d.ldc, d.c_bstride = C.data_ptr() + 4 * c_off, ldc, c_bstride
    d.alpha, d.beta = alpha, beta
    d.bias, d.bias_mode, d.act = (bias.data_ptr() if bias is not None else None), bias_mode, act
    d.aux, d.ldaux, d.aux_bstride = (aux.data_ptr() if aux is not None else None), ldaux, aux_bstride
    d.residual, d.ldres, d.res_bstride = (residual.data_ptr() if residual is not None else None), ldres, res_bstride
    d.split_k = split_k if split_k is not None else _split_for(M, N, K)
    if conv is not None:
        d.conv = conv
    if preact is not None:
        d.preact, d.ldpre, d.pre_bstride = preact.data_ptr(), ldpre, pre_bstride
    if rowsum_a is not None:
        d.rowsum_a = rowsum_a.data_ptr()
    if row_scale is not None:
        d.row_scale, d.row_scale_group = row_scale.data_ptr(), row_scale_group
    lib = L.load()
    need = lib.mdemi_gemm_workspace_size(ctypes.byref(d))
    if need:
        ws = L.workspace(need, C.device, slot=1)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
    if (_PRECISION[0] == "bf16" and _B16_STORAGE[0] and a16 is None and b16 is None and a_op == L.OP_NONE
            and b_op == L.OP_NONE and A is not None and B is not None):
        a16, b16 = _b16_operands(d, A, B, a_off, b_off, rowsum_a, lib)
        if a16 is not None and rowsum_a is not None and (a_layout != L.L_MNCONTIG or batch != 1):
            # the column-sum substitution below assumes an m-contiguous [K][M] A of batch 1
            # (mdemi_gemm_desc.rowsum_a's own contract): anything else keeps the in-kernel
            # sums on the fp32-operand path
            a16 = b16 = None
        if a16 is not None and rowsum_a is not None:
            # the bias-gradient row sums of the unrounded fp32 A: a column sum over A's k rows
            # (A m-contiguous [K][M]), instead of the GEMM's in-kernel sums
            ws = L.workspace(lib.mdemi_colsum_workspace_size(K, M), C.device, slot=2)
            L.check(lib.mdemi_colsum_f32(A.data_ptr() + 4 * a_off, K, M, lda, rowsum_a.data_ptr(), 0, ws.data_ptr(),
                                         L.stream()), "colsum")
            d.rowsum_a = None
            need = lib.mdemi_gemm_workspace_size(ctypes.byref(d))
            if need:
                ws = L.workspace(need, C.device, slot=1)
                d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
    if (A is None or B is None) and not lib.mdemi_gemm_bf16x_supported(
            ctypes.byref(d), None if a16 is None else a16.data_ptr() + 2 * a_off,
            None if b16 is None else b16.data_ptr() + 2 * b_off):
        raise B16Unsupported("gemm: no bf16 path for this layout and no fp32 operand to fall back on")
    LAST_GEMM[0] = "b16" if (a16 is not None and b16 is not None) else _PRECISION[0]
    if a16 is not None or b16 is not None or c16 is not None:
        if _PRECISION[0] != "bf16":
            raise ValueError("gemm: bf16 operands / output (a16, b16, c16) need matmul precision 'bf16'")
        L.check(lib.mdemi_gemm_bf16x(ctypes.byref(d), None if a16 is None else a16.data_ptr() + 2 * a_off,
                                     None if b16 is None else b16.data_ptr() + 2 * b_off,
                                     None if c16 is None else c16.data_ptr() + 2 * c_off, L.stream()), "gemm_bf16x")
    elif _PRECISION[0] == "bf16":
        L.check(lib.mdemi_gemm_bf16(ctypes.byref(d), L.stream()), "gemm_bf16")
    elif _PRECISION[0] == "fp32e":
        L.check(lib.mdemi_gemm_f32e(ctypes.byref(d), L.stream()), "gemm_f32e")
    else:
        L.check(lib.mdemi_gemm_f32(ctypes.byref(d), L.stream()), "gemm_f32")
    return C


class B16Unsupported(RuntimeError):
    """gemm() given only the bf16 copy of an operand whose layout the bf16 loaders cannot stage
    (what mdemi_gemm_bf16x itself refuses with "no bf16 path"), raised before any launch."""


def _b16_operands(d, A, B, a_off, b_off, rowsum_a, lib):
    """(a16, b16) for a bf16 GEMM the bf16-operand kernel can run (bf16 storage on), else
    (None, None).  The layout check runs on the fp32 descriptor before any copy is made."""
    for t in (A, B):
        if not t.is_contiguous() or t.data_ptr() % 16:
            return None, None
    if a_off % 8 or b_off % 8:  # the bf16 slices must start 16-B aligned
        return None, None
    rs = d.rowsum_a
    d.rowsum_a = None  # the row sums are taken by a column sum instead (gemm)
    ok = lib.mdemi_gemm_bf16x_supported(ctypes.byref(d), A.data_ptr(), B.data_ptr())
    d.rowsum_a = rs
    if not ok:
        return None, None
    a16, b16 = b16_of(A), b16_of(B)
    if a16 is None or b16 is None:
        return None, None
    return a16, b16


def colsum(x2d, out=None, accumulate=False):
    rows, cols = x2d.shape
    if out is None:
        out = torch.empty(cols, device=x2d.device, dtype=torch.float32)
    lib = L.load()
    ws = L.workspace(lib.mdemi_colsum_workspace_size(rows, cols), x2d.device)
    L.check(lib.mdemi_colsum_f32(x2d.data_ptr(), rows, cols, x2d.stride(0), out.data_ptr(), int(accumulate),
                                 ws.data_ptr(), L.stream()), "colsum")
    return out


# --------------------------------------------------------------------------
# Linear (nn.Linear) with GELU-on-load input and fused residual
# --------------------------------------------------------------------------


def linear_fwd_raw(x2, weight, bias, in_gelu=False, residual=None, act=L.ACT_NONE, out=None, drop_scale=None,
                   c16=None):
    """drop_scale: per-sample DropPath scale [B] of the product (rows grouped M / B per sample),
    applied in the epilogue before the residual add; c16: the output's bf16 copy (gemm())."""
    M, K = x2.shape
    N = weight.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x2.device, dtype=torch.float32)
    gemm(x2, weight, out, M, N, K, lda=K, ldb=K, ldc=out.stride(0), a_layout=L.L_KCONTIG,
         b_layout=L.L_KCONTIG, a_op=L.OP_GELU if in_gelu else L.OP_NONE,
         bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, act=act,
         residual=residual, ldres=(residual.stride(0) if residual is not None else 0), split_k=1,
         row_scale=drop_scale, row_scale_group=(M // drop_scale.numel() if drop_scale is not None else 0),
         c16=c16)
    return out


def _drop_rows(dy2, scale):
    """s[sample] * dy: the DropPath branch gradient (rows grouped per sample)."""
    db = torch.empty_like(dy2)
    L.call("mdemi_rowscale_add", None, dy2.data_ptr(), scale.data_ptr(), db.data_ptr(), dy2.numel() // scale.numel(),
           dy2.numel(), L.stream())
    return db


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, in_gelu, drop_scale, out_b16=False):
        _require_cuda(x, weight, bias, residual)
        K = x.shape[-1]
        x2 = _c(x).reshape(-1, K)
        res2 = _c(residual).reshape(x2.shape[0], -1) if residual is not None else None
        out = torch.empty(x2.shape[0], weight.shape[0], device=x.device, dtype=torch.float32)
        o16 = new_b16_like(out) if out_b16 else None  # the output feeds bf16 GEMMs (attention products)
        linear_fwd_raw(x2, _c(weight), bias, in_gelu=in_gelu, residual=res2, drop_scale=drop_scale, out=out, c16=o16)
        if o16 is not None:
            set_b16(out, o16)
        ctx.save_for_backward(x2, weight)
        ctx.dx16 = grad_feeds_gemm(x)
        ctx.drop_scale = drop_scale
        ctx.in_gelu = in_gelu
        ctx.has_bias = bias is not None
        ctx.has_res = residual is not None
        ctx.xshape = x.shape
        return out.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        M, K = x2.shape
        N = weight.shape[0]
        dy2 = _c(dy).reshape(M, N)
        if ctx.drop_scale is not None:  # the branch's gradient; the residual's stays dy
            dy2 = _drop_rows(dy2, ctx.drop_scale)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dy.device, dtype=torch.float32)
            dx16 = new_b16_like(dx) if ctx.dx16 else None  # dX is the next GEMM backward's operand
            # dX[M,K] = dY[M,N] . W[N,K]  (times gelu'(h) when the forward read gelu(h))
            gemm(dy2, weight, dx, M, K, N, lda=N, ldb=K, ldc=K, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG,
                 act=L.ACT_GELU_GRAD if ctx.in_gelu else L.ACT_NONE, aux=x2 if ctx.in_gelu else None,
                 ldaux=K, c16=dx16)
            if dx16 is not None:
                set_b16(dx, dx16)
            dx = dx.view(ctx.xshape)
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        if want_db:
            db = torch.empty(N, device=dy.device, dtype=torch.float32)
        if ctx.needs_input_grad[1]:
            dw = torch.empty(N, K, device=dy.device, dtype=torch.float32)
            # dW[N,K] = dY^T . X  (reduction over the M rows; split-K slabs); db = dY^T 1 rides along
            gemm(dy2, x2, dw, N, K, M, lda=N, ldb=K, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                 b_op=L.OP_GELU if ctx.in_gelu else L.OP_NONE, rowsum_a=db)
        elif want_db:
            colsum(dy2, out=db)
        dres = dy if ctx.has_res and ctx.needs_input_grad[3] else None
        return dx, dw, db, dres, None, None, None


def linear(x, weight, bias=None, residual=None, in_gelu=False, drop_scale=None, p=0.0, training=False,
           out_b16=False):
    """y = (gelu(x) if in_gelu else x) @ W^T + b (+ residual); drop_scale (DropPath, per
    sample [B]): y = residual + drop_scale[sample] * (x @ W^T + b), fused in the epilogue.
    p > 0 and training: y = dropout(x @ W^T + b) (+ residual) -- nn.Dropout on a projection's
    output before a residual add (luna_layer.py:172-173,250-251, self_attention.py:78-80); the
    residual add is then a separate sweep after the dropout one.  out_b16 (no dropout): the
    output's bf16 copy from the epilogue, for bf16 GEMMs that read it (bf16 storage)."""
    if drop_scale is not None and residual is None:
        raise ValueError("linear: drop_scale scales a residual branch and needs residual")
    if training and p > 0.0:
        if drop_scale is not None:
            raise ValueError("linear: dropout and drop_scale together are not supported")
        y = dropout(_LinearFn.apply(x, weight, bias, None, in_gelu, None, False), p, True)
        return add(residual, y) if residual is not None else y
    return _LinearFn.apply(x, weight, bias, residual, in_gelu, drop_scale, out_b16)


class _MlpFn(torch.autograd.Function):
    """fc1 -> act -> [dropout] -> fc2 -> [dropout] (+ residual): Swin/NeW-CRF Mlp
    (swin_transformer.py:11-29, GELU), Depthformer FeedForwardBlock (feed_forward.py:29-46,
    SiLU) and nn.TransformerEncoderLayer's feed-forward (layers.py:8, ReLU).

    fc1's epilogue writes both h (pre-activation) and g = act(h): HBM is
    plentiful and one extra [rows, 4C] store is far cheaper than recomputing
    act in fc2's operand loader for every N-tile.  Backward without dropout:
    fc2's dgrad epilogue multiplies by act'(h) (reading h), so dh never exists
    unfused.  Dropout masks are counter hashes regenerated in the backward."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual, cfg):
        act, p_mid, p_out, seed, drop_scale = cfg
        _require_cuda(x, w1, b1, w2, b2, residual)
        K = x.shape[-1]
        x2 = _c(x).reshape(-1, K)
        M = x2.shape[0]
        Hd, N = w1.shape[0], w2.shape[0]
        h = torch.empty(M, Hd, device=x.device, dtype=torch.float32)
        g = torch.empty(M, Hd, device=x.device, dtype=torch.float32)
        g16 = new_b16_like(g) if g.numel() % 4 == 0 else None  # fc2's operand (bf16 storage)
        gemm(x2, _c(w1), g, M, Hd, K, lda=K, ldb=K, ldc=Hd, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
             bias=b1, bias_mode=L.BIAS_COL if b1 is not None else L.BIAS_NONE, act=act,
             preact=h, ldpre=Hd, split_k=1, c16=g16 if p_mid == 0.0 else None)
        if p_mid > 0.0:
            _drop(g.data_ptr(), g.data_ptr(), g.numel(), p_mid, seed, dst16_ptr=L.ptr(g16))
        if g16 is not None:
            set_b16(g, g16)
        res2 = _c(residual).reshape(M, N) if residual is not None else None
        if p_out > 0.0:
            out = linear_fwd_raw(g, _c(w2), b2)
            _drop(out.data_ptr(), out.data_ptr(), out.numel(), p_out, seed, add=1)
            if res2 is not None:
                L.call("mdemi_elementwise", L.EW_ADD, out.data_ptr(), res2.data_ptr(), out.data_ptr(), out.numel(),
                       0.0, 0.0, L.stream())
        else:
            out = linear_fwd_raw(g, _c(w2), b2, residual=res2, drop_scale=drop_scale)
        ctx.save_for_backward(x2, w1, w2, h, g)
        ctx.flags = (b1 is not None, b2 is not None, residual is not None)
        ctx.cfg = cfg
        ctx.xshape = x.shape
        return out.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w1, w2, h, g = ctx.saved_tensors
        has_b1, has_b2, has_res = ctx.flags
        act, p_mid, p_out, seed, drop_scale = ctx.cfg
        M, K = x2.shape
        Hd, N = w1.shape[0], w2.shape[0]
        dy2 = _c(dy).reshape(M, N)
        if drop_scale is not None:  # the branch's gradient; the residual's stays dy
            dy2 = _drop_rows(dy2, drop_scale)
        dev = dy.device
        if p_out > 0.0:
            d2 = torch.empty_like(dy2)
            d216 = new_b16_like(d2) if d2.numel() % 4 == 0 and dy2.data_ptr() % 16 == 0 else None
            _drop(dy2.data_ptr(), d2.data_ptr(), d2.numel(), p_out, seed, add=1, dst16_ptr=L.ptr(d216))
            if d216 is not None:
                set_b16(d2, d216)  # the operand of both fc2 gradient GEMMs
        else:
            d2 = dy2
        dw2 = torch.empty(N, Hd, device=dev, dtype=torch.float32)
        db2 = torch.empty(N, device=dev, dtype=torch.float32) if has_b2 else None
        gemm(d2, g, dw2, N, Hd, M, lda=N, ldb=Hd, ldc=Hd, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             rowsum_a=db2)
        dh = torch.empty(M, Hd, device=dev, dtype=torch.float32)
        if p_mid > 0.0:
            gemm(d2, w2, dh, M, Hd, N, lda=N, ldb=Hd, ldc=Hd, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
            _drop(dh.data_ptr(), dh.data_ptr(), dh.numel(), p_mid, seed)
            L.call("mdemi_elementwise", L.EW_ACT_BWD, h.data_ptr(), dh.data_ptr(), dh.data_ptr(), dh.numel(),
                   float(act), 0.0, L.stream())
        else:
            dh16 = new_b16_like(dh)  # the operand of both fc1 gradient GEMMs
            gemm(d2, w2, dh, M, Hd, N, lda=N, ldb=Hd, ldc=Hd, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG,
                 act=L.ACT_GRAD_OF[act], aux=h, ldaux=Hd, c16=dh16)
            if dh16 is not None:
                set_b16(dh, dh16)
        del h, g
        dw1 = torch.empty(Hd, K, device=dev, dtype=torch.float32)
        db1 = torch.empty(Hd, device=dev, dtype=torch.float32) if has_b1 else None
        gemm(dh, x2, dw1, Hd, K, M, lda=Hd, ldb=K, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             rowsum_a=db1)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dev, dtype=torch.float32)
            gemm(dh, w1, dx, M, K, Hd, lda=Hd, ldb=K, ldc=K, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
            dx = dx.view(ctx.xshape)
        dres = dy if has_res and ctx.needs_input_grad[5] else None
        return dx, dw1, db1, dw2, db2, dres, None


def mlp(x, w1, b1, w2, b2, residual=None, act=L.ACT_GELU, p_mid=0.0, p_out=0.0, training=False, drop_scale=None):
    """fc2(dropout(act(fc1(x)))) -> dropout (+ residual); act GELU (exact erf), SiLU or ReLU.
    drop_scale (DropPath, per sample [B]): residual + drop_scale[sample] * branch, fused in
    fc2's epilogue (no output dropout with it)."""
    if not training:
        p_mid = p_out = 0.0
    if drop_scale is not None and (residual is None or p_out > 0.0):
        raise ValueError("mlp: drop_scale needs a residual and no output dropout")
    seed = _draw_seed(x.device) if (p_mid > 0.0 or p_out > 0.0) else None
    return _MlpFn.apply(x, w1, b1, w2, b2, residual, (act, float(p_mid), float(p_out), seed, drop_scale))


# --------------------------------------------------------------------------
# Conv2d on NHWC activations (implicit im2col on the GEMM operand loader)
# --------------------------------------------------------------------------


def _geom(n, h, w, c, oh, ow, kh, kw, stride, pad, pad_mode):
    g = L.ConvGeom()
    g.n, g.h, g.w, g.c, g.oh, g.ow = n, h, w, c, oh, ow
    g.kh, g.kw, g.stride, g.pad, g.pad_mode = kh, kw, stride, pad, pad_mode
    return g


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, pad_mode, act, out_hw=None):
        _require_cuda(x, weight, bias)
        x = _c(x)
        n, h, w, c = x.shape
        cout, cin, kh, kw = weight.shape
        if cin != c:
            raise ValueError(f"conv2d: input has {c} channels, weight expects {cin}")
        if out_hw is None:
            oh = (h + 2 * pad - kh) // stride + 1
            ow = (w + 2 * pad - kw) // stride + 1
        else:  # explicit output size: `pad` is the top/left padding (TF 'same', asymmetric)
            oh, ow = out_hw
        M, K = n * oh * ow, kh * kw * c
        out = torch.empty(n, oh, ow, cout, device=x.device, dtype=torch.float32)
        wf = conv_weight_layout(weight, L.WL_OHWI).view(cout, K)
        pointwise = kh == 1 and kw == 1 and stride == 1 and pad == 0
        if pointwise:
            # bf16: the split-K heuristic too -- the 15x20 / 30x40 EfficientNet projections have
            # 57-400 output tiles over K up to 3072, and the bf16 families combine slabs with a
            # parallel reduce kernel (gemm_f32.hip g_inline_reduce_b16)
            gemm(x, wf, out, M, cout, K, lda=c, ldb=K, ldc=cout, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
                 bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, act=act,
                 split_k=None if _PRECISION[0] == "bf16" else 1)
        else:
            if c % 4:
                raise ValueError("conv2d: implicit-GEMM path needs C % 4 == 0")
            gemm(x, wf, out, M, cout, K, lda=0, ldb=K, ldc=cout, a_layout=L.L_CONV, b_layout=L.L_KCONTIG,
                 bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, act=act,
                 conv=_geom(n, h, w, c, oh, ow, kh, kw, stride, pad, pad_mode))
        ctx.save_for_backward(x, weight, out if act != L.ACT_NONE else None)
        ctx.cfg = (stride, pad, pad_mode, act, bias is not None, pointwise)
        ctx.explicit = out_hw is not None
        return out

    @staticmethod
    def backward(ctx, dy):
        return _conv2d_backward(ctx, dy, None)


def _conv2d_backward(ctx, dy, dskip):
    """_Conv2dFn's backward; dskip (pointwise only): the gradient of the conv's input through a
    residual skip, added in the input-gradient GEMM's epilogue."""
    x, weight, y = ctx.saved_tensors
    stride, pad, pad_mode, act, has_bias, pointwise = ctx.cfg
    dy = _c(dy)
    if act != L.ACT_NONE:
        if act != L.ACT_RELU:
            raise NotImplementedError("conv2d backward: only ReLU epilogue supported")
        g = torch.empty_like(dy)
        L.call("mdemi_elementwise", L.EW_ACT_BWD, y.data_ptr(), dy.data_ptr(), g.data_ptr(), dy.numel(),
               float(L.ACT_RELU), 0.0, L.stream())
        dy = g
    n, h, w, c = x.shape
    cout, cin, kh, kw = weight.shape
    _, oh, ow, _ = dy.shape
    M, K = n * oh * ow, kh * kw * c
    dx = dw = db = None
    if ctx.needs_input_grad[0]:
        if pointwise:
            dx = torch.empty_like(x)
            gemm(dy, weight.reshape(cout, cin), dx, M, c, cout, lda=cout, ldb=cin, ldc=c,
                 a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG, residual=dskip, ldres=c if dskip is not None else 0)
        elif dskip is not None:
            raise NotImplementedError("conv2d skip: pointwise convs only")
        elif stride == kh == kw and pad == 0 and not ctx.explicit:
            # non-overlapping patches (mViT embedding_encoder): column gradients by one GEMM
            # against the (ky,kx,c)-ordered weight, then a scatter back to the NHWC pixels
            wf = conv_weight_layout(weight, L.WL_OHWI).view(cout, K)
            dcols = torch.empty(M, K, device=dy.device, dtype=torch.float32)
            gemm(dy, wf, dcols, M, K, cout, lda=cout, ldb=K, ldc=K, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
            dx = torch.empty_like(x)
            L.call("mdemi_unpatchify_nhwc", dcols.data_ptr(), dx.data_ptr(), n, h, w, c, stride, oh, ow,
                   L.stream())
        else:
            if stride != 1 or ctx.explicit:
                raise NotImplementedError("conv2d dgrad: stride 1 or stride == kernel only")
            # dX = conv(dY, flip(W)^T) with pad k-1-p:  Wd[(ky,kx,co)][c] = W[co][c][k-1-ky][k-1-kx]
            wd = conv_weight_layout(weight, L.WL_DGRAD).view(kh * kw * cout, cin)
            dx = torch.empty_like(x)
            if pad_mode == L.PAD_ZERO:
                gemm(dy, wd, dx, n * h * w, c, kh * kw * cout, lda=0, ldb=cin, ldc=c, a_layout=L.L_CONV,
                     b_layout=L.L_MNCONTIG,
                     conv=_geom(n, oh, ow, cout, h, w, kh, kw, 1, kh - 1 - pad, L.PAD_ZERO))
            else:
                # replicate padding (layer_utils.py:21): gradient of the padded input by a full
                # correlation, then fold the border rows/columns onto the edge pixels
                hp, wp = h + 2 * pad, w + 2 * pad
                dxp = torch.empty(n, hp, wp, c, device=dy.device, dtype=torch.float32)
                gemm(dy, wd, dxp, n * hp * wp, c, kh * kw * cout, lda=0, ldb=cin, ldc=c, a_layout=L.L_CONV,
                     b_layout=L.L_MNCONTIG,
                     conv=_geom(n, oh, ow, cout, hp, wp, kh, kw, 1, kh - 1, L.PAD_ZERO))
                L.call("mdemi_pad_fold_replicate", dxp.data_ptr(), dx.data_ptr(), n, h, w, c, pad, L.stream())
    want_db = has_bias and ctx.needs_input_grad[2]
    if want_db:
        db = torch.empty(cout, device=dy.device, dtype=torch.float32)
    if ctx.needs_input_grad[1]:
        dwf = torch.empty(cout, K, device=dy.device, dtype=torch.float32)
        if pointwise:
            gemm(dy, x, dwf, cout, K, M, lda=cout, ldb=c, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                 rowsum_a=db)
        else:
            gemm(dy, x, dwf, cout, K, M, lda=cout, ldb=0, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_CONV,
                 conv=_geom(n, h, w, c, oh, ow, kh, kw, stride, pad, pad_mode), rowsum_a=db)
        dw = conv_weight_layout(dwf, L.WL_OIHW, (cout, cin, kh, kw))
    elif want_db:
        colsum(dy.reshape(-1, cout), out=db)
    return dx, dw, db, None, None, None, None, None


class _Conv2dSkipFn(torch.autograd.Function):
    """x -> (conv1x1(x), x): a pointwise conv whose input is also its block's residual
    (EfficientNet InvertedResidual: conv_pw(x) ... + x, gen-efficientnet via
    unet_adaptive_bins.py:129 / depthformer_v8.py:89).  The two gradient contributions to x meet
    in the input-gradient GEMM's epilogue (residual = the skip's gradient) instead of an autograd
    add over the block input; the sum is the same fp32 addition, so results are unchanged."""

    @staticmethod
    def forward(ctx, x, weight):
        out = _Conv2dFn.forward(ctx, x, weight, None, 1, 0, L.PAD_ZERO, L.ACT_NONE)
        ctx.set_materialize_grads(False)
        return out, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        if dy is None:
            return dskip, None
        dskip = _c(dskip) if dskip is not None else None
        dx, dw, _ = _conv2d_backward(ctx, dy, dskip)[:3]
        return dx, dw


# MDEMI_CONV_SKIP=0: the autograd add instead (A/B and the bit-identity test)
_FUSE_SKIP = [os.environ.get("MDEMI_CONV_SKIP", "1") != "0"]


def conv2d_nhwc_skip(x, weight):
    """(conv1x1(x), x) for a residual block whose first op is a bias-free pointwise conv: use the
    second output as the block's skip, so the input gradient is one GEMM epilogue."""
    if weight.shape[-1] != 1 or weight.shape[-2] != 1:
        raise ValueError("conv2d_nhwc_skip: pointwise (1x1) convs only")
    if not _FUSE_SKIP[0]:
        return _Conv2dFn.apply(x, weight, None, 1, 0, L.PAD_ZERO, L.ACT_NONE), x
    return _Conv2dSkipFn.apply(x, weight)


class _HeadConvFn(torch.autograd.Function):
    """KxK 'same' conv with a single output channel (DispHead.conv1)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        _require_cuda(x, weight, bias)
        x, weight = _c(x), _c(weight)
        n, h, w, c = x.shape
        k = weight.shape[-1]
        y = torch.empty(n, h, w, 1, device=x.device, dtype=torch.float32)
        L.call("mdemi_headconv_fwd", x.data_ptr(), weight.data_ptr(), L.ptr(bias), y.data_ptr(), n, h, w, c, k,
               k // 2, L.stream())
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = _c(dy)
        n, h, w, c = x.shape
        k = weight.shape[-1]
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(weight) if ctx.needs_input_grad[1] else None
        db = torch.empty(1, device=x.device, dtype=torch.float32) if ctx.has_bias and ctx.needs_input_grad[2] else None
        lib = L.load()
        ws = L.workspace(lib.mdemi_headconv_wgrad_workspace_size(n, h, w, c, k), x.device)
        L.check(lib.mdemi_headconv_bwd(dy.data_ptr(), x.data_ptr(), weight.data_ptr(), L.ptr(dx), L.ptr(dw), L.ptr(db),
                                       n, h, w, c, k, k // 2, ws.data_ptr(), L.stream()), "headconv_bwd")
        return dx, dw, db


def conv2d_nhwc(x, weight, bias=None, stride=1, pad=0, pad_mode=L.PAD_ZERO, act=L.ACT_NONE, out_hw=None):
    if out_hw is not None:
        return _Conv2dFn.apply(x, weight, bias, stride, pad, pad_mode, act, tuple(out_hw))
    if weight.shape[0] == 1 and stride == 1 and pad_mode == L.PAD_ZERO and act == L.ACT_NONE and \
            2 * pad == weight.shape[-1] - 1 and weight.shape[-1] <= 3 and x.shape[-1] % 4 == 0 and \
            x.shape[-1] <= 128:
        return _HeadConvFn.apply(x, weight, bias)
    return _Conv2dFn.apply(x, weight, bias, stride, pad, pad_mode, act)


class _PatchEmbedFn(torch.autograd.Function):
    """Conv with kernel == stride (PatchEmbed, swin_transformer.py:414,429) on an NCHW image:
    patchify sweep + GEMM.  Output NHWC.  The image gets no gradient."""

    @staticmethod
    def forward(ctx, img, weight, bias):
        _require_cuda(img, weight, bias)
        img = _c(img)
        n, c, h, w = img.shape
        cout, cin, p, _ = weight.shape
        hp, wp = -(-h // p), -(-w // p)
        K = c * p * p
        cols = torch.empty(n * hp * wp, K, device=img.device, dtype=torch.float32)
        L.call("mdemi_patchify_nchw", img.data_ptr(), cols.data_ptr(), n, c, h, w, p, 0, L.stream())
        out = torch.empty(n, hp, wp, cout, device=img.device, dtype=torch.float32)
        gemm(cols, _c(weight).reshape(cout, K), out, n * hp * wp, cout, K, lda=K, ldb=K, ldc=cout,
             a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG, bias=bias,
             bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, split_k=1)
        ctx.save_for_backward(cols, weight)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, dy):
        cols, weight = ctx.saved_tensors
        cout = weight.shape[0]
        M, K = cols.shape
        dy2 = _c(dy).reshape(M, cout)
        dw = torch.empty(cout, K, device=dy.device, dtype=torch.float32)
        db = torch.empty(cout, device=dy.device, dtype=torch.float32) if ctx.has_bias else None
        gemm(dy2, cols, dw, cout, K, M, lda=cout, ldb=K, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             rowsum_a=db)
        return None, dw.view_as(weight), db


def patch_embed(img_nchw, weight, bias):
    return _PatchEmbedFn.apply(img_nchw, weight, bias)


# --------------------------------------------------------------------------
# LayerNorm
# --------------------------------------------------------------------------


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_b16=False):
        """out_b16: y feeds a bf16 GEMM -- write its bf16 copy in the same sweep (bf16 storage)."""
        _require_cuda(x, weight, bias)
        x = _c(x)
        C = x.shape[-1]
        rows = x.numel() // C
        y = torch.empty_like(x)
        y16 = new_b16_like(y) if out_b16 else None
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        L.call("mdemi_layernorm_fwd16", x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(), L.ptr(y16),
               mean.data_ptr(), rstd.data_ptr(), rows, C, float(eps), L.stream())
        if y16 is not None:
            set_b16(y, y16)
        ctx.save_for_backward(x, weight, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, rstd = ctx.saved_tensors
        dy = _c(dy)
        C = x.shape[-1]
        rows = x.numel() // C
        dx = torch.empty_like(x)
        dg = torch.empty(C, device=x.device, dtype=torch.float32)
        db = torch.empty(C, device=x.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_layernorm_bwd_workspace_size(rows, C), x.device)
        L.check(lib.mdemi_layernorm_bwd(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                        weight.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), rows, C, 0,
                                        ws.data_ptr(), L.stream()), "layernorm_bwd")
        return dx, dg, db, None, None


class _LayerNormSkipFn(torch.autograd.Function):
    """x -> (LayerNorm(x), x): a LayerNorm whose input is also the block's residual.  The two
    gradient contributions to x meet inside the LayerNorm backward sweep
    (mdemi_layernorm_bwd_add) instead of an extra elementwise add of autograd."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, out_b16=False):
        _require_cuda(x, weight, bias)
        x = _c(x)
        C = x.shape[-1]
        rows = x.numel() // C
        y = torch.empty_like(x)
        y16 = new_b16_like(y) if out_b16 else None  # LN(x) feeds a bf16 GEMM (bf16 storage)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        L.call("mdemi_layernorm_fwd16", x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(), L.ptr(y16),
               mean.data_ptr(), rstd.data_ptr(), rows, C, float(eps), L.stream())
        if y16 is not None:
            set_b16(y, y16)
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.set_materialize_grads(False)  # an unused output's gradient stays None (no zero fill)
        skip = x.view_as(x)
        return y, skip

    @staticmethod
    def backward(ctx, dy, dskip):
        x, weight, mean, rstd = ctx.saved_tensors
        C = x.shape[-1]
        rows = x.numel() // C
        dx = torch.empty_like(x)
        dg = torch.empty(C, device=x.device, dtype=torch.float32)
        db = torch.empty(C, device=x.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_layernorm_bwd_workspace_size(rows, C), x.device)
        if dy is None:
            return dskip, None, None, None, None
        dy = _c(dy)
        if dskip is None:
            L.check(lib.mdemi_layernorm_bwd(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                            weight.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), rows, C,
                                            0, ws.data_ptr(), L.stream()), "layernorm_bwd")
        else:
            dskip = _c(dskip)
            L.check(lib.mdemi_layernorm_bwd_add(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                                weight.data_ptr(), dskip.data_ptr(), dx.data_ptr(), dg.data_ptr(),
                                                db.data_ptr(), rows, C, ws.data_ptr(), L.stream()), "layernorm_bwd_add")
        return dx, dg, db, None, None


def layer_norm_skip(x, weight, bias, eps=1e-5, out_b16=False):
    """(LayerNorm(x), x) for a residual block; use the second output as the residual.
    out_b16: LayerNorm(x) feeds a bf16 GEMM (bf16 storage writes its bf16 copy too)."""
    return _LayerNormSkipFn.apply(x, weight, bias, eps, out_b16)


def layer_norm(x, weight, bias, eps=1e-5, out_b16=False):
    """out_b16: the output feeds a bf16 GEMM (bf16 storage writes its bf16 copy too)."""
    return _LayerNormFn.apply(x, weight, bias, eps, out_b16)


# --------------------------------------------------------------------------
# (Shifted-)window attention
# --------------------------------------------------------------------------


class _WindowAttnFn(torch.autograd.Function):
    """q/k come from `qk` ([rows, >=2C]: q at col 0, k at col C); v from `v` ([rows, ...] at
    column v_off).  Pad tokens read qk_bias / v_bias (None -> zeros)."""

    @staticmethod
    def forward(ctx, qk, qk_bias, v, v_bias, rpb, geom):
        _require_cuda(qk, qk_bias, v, v_bias, rpb)
        B, H, W, heads, window, shift, scale, C, v_off = geom
        rows = B * H * W
        out = torch.empty(rows, C, device=qk.device, dtype=torch.float32)
        d = L.WinAttnDesc()
        d.B, d.H, d.W, d.heads, d.head_dim, d.window, d.shift = B, H, W, heads, C // heads, window, shift
        d.scale = scale
        d.q, d.k, d.qk_ld = qk.data_ptr(), qk.data_ptr() + 4 * C, qk.stride(0)
        d.q_pad = qk_bias.data_ptr() if qk_bias is not None else None
        d.k_pad = qk_bias.data_ptr() + 4 * C if qk_bias is not None else None
        d.v, d.v_ld = v.data_ptr() + 4 * v_off, v.stride(0)
        d.v_pad = v_bias.data_ptr() + 4 * v_off if v_bias is not None else None
        d.rpb_table = rpb.data_ptr()
        d.out, d.out_ld = out.data_ptr(), C
        ws = window
        nwin = B * (-(-H // ws)) * (-(-W // ws))
        lse = torch.empty(nwin, heads, ws * ws, device=qk.device, dtype=torch.float32)
        d.lse = lse.data_ptr()
        lib = L.load()
        # the forward's workspace is the expanded relative-position bias: a buffer of this call's
        # own (heads x 16 KiB), kept for the backward instead of expanding the table again
        bias_x = torch.empty(lib.mdemi_winattn_fwd_workspace_size(ctypes.byref(d)) // 4, device=qk.device,
                             dtype=torch.float32)
        d.workspace, d.workspace_bytes = bias_x.data_ptr(), 4 * bias_x.numel()
        L.check(lib.mdemi_winattn_fwd(ctypes.byref(d), L.stream()), "winattn_fwd")
        ctx.bias_x = bias_x
        ctx.rpb_version = rpb._version
        ctx.save_for_backward(qk, qk_bias, v, v_bias, rpb, out, lse)
        ctx.geom = geom
        ctx.has_qkb = qk_bias is not None
        ctx.has_vb = v_bias is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        qk, qk_bias, v, v_bias, rpb, out, lse = ctx.saved_tensors
        B, H, W, heads, window, shift, scale, C, v_off = ctx.geom
        dout = _c(dout)
        dqk = torch.empty_like(qk)
        same = v.data_ptr() == qk.data_ptr()
        if same:
            dv_t = dqk
        else:
            dv_t = torch.empty_like(v)
        if dqk.shape[1] > 2 * C and not same:
            dqk[:, 2 * C:].zero_()
        if dv_t.shape[1] > C and not same:
            dv_t.zero_()
        d_rpb = torch.empty_like(rpb)
        # the pad tokens' (q, k, v) gradients, which the kernel's scatter writes whole (dq: zeros):
        # straight into the bias gradients where their layout allows (Swin qkv.bias [q|k|v];
        # NeW-CRF qk.bias [q|k] with a bias-free v), else into a [3, C] scratch assembled below
        dqk_bias = dv_bias = None
        if ctx.has_qkb and same and ctx.has_vb and v_off == 2 * C and qk_bias.numel() == 3 * C:
            dqk_bias = torch.empty_like(qk_bias)
            pad_g = dqk_bias.view(3, C)
        elif ctx.has_qkb and not same and not ctx.has_vb and qk_bias.numel() == 2 * C:
            dqk_bias = torch.empty_like(qk_bias)
            pad_g = (dqk_bias[:C], dqk_bias[C:], torch.empty(C, device=qk.device, dtype=torch.float32))
        else:
            pad_g = torch.empty(3, C, device=qk.device, dtype=torch.float32)
        d = L.WinAttnDesc()
        d.B, d.H, d.W, d.heads, d.head_dim, d.window, d.shift = B, H, W, heads, C // heads, window, shift
        d.scale = scale
        d.q, d.k, d.qk_ld = qk.data_ptr(), qk.data_ptr() + 4 * C, qk.stride(0)
        d.q_pad = qk_bias.data_ptr() if qk_bias is not None else None
        d.k_pad = qk_bias.data_ptr() + 4 * C if qk_bias is not None else None
        d.v, d.v_ld = v.data_ptr() + 4 * v_off, v.stride(0)
        d.v_pad = v_bias.data_ptr() + 4 * v_off if v_bias is not None else None
        d.rpb_table = rpb.data_ptr()
        d.out, d.out_ld, d.lse = out.data_ptr(), C, lse.data_ptr()
        d.dout = dout.data_ptr()
        d.dq, d.dk, d.dqk_ld = dqk.data_ptr(), dqk.data_ptr() + 4 * C, dqk.stride(0)
        d.dv, d.dv_ld = dv_t.data_ptr() + 4 * v_off, dv_t.stride(0)
        d.d_rpb_table = d_rpb.data_ptr()
        d.dq_pad, d.dk_pad, d.dv_pad = pad_g[0].data_ptr(), pad_g[1].data_ptr(), pad_g[2].data_ptr()
        lib = L.load()
        need = lib.mdemi_winattn_bwd_workspace_size(ctypes.byref(d))
        ws = L.workspace(need, qk.device)
        d.workspace, d.workspace_bytes = ws.data_ptr(), ws.numel()
        # the forward's expansion is valid while the table is unchanged (no in-place update since)
        bias_x = ctx.bias_x if rpb._version == ctx.rpb_version else None
        L.check(lib.mdemi_winattn_bwd_bias(ctypes.byref(d), L.ptr(bias_x), L.stream()), "winattn_bwd")
        if ctx.has_qkb and dqk_bias is None:
            dqk_bias = torch.zeros_like(qk_bias)
            dqk_bias[:C] = pad_g[0]
            dqk_bias[C:2 * C] = pad_g[1]
            if same and ctx.has_vb:
                dqk_bias[v_off:v_off + C] += pad_g[2]
        if ctx.has_vb and not same:
            dv_bias = torch.zeros_like(v_bias)
            dv_bias[v_off:v_off + C] = pad_g[2]
        if same:
            return dqk, dqk_bias, None, None, d_rpb, None
        return dqk, dqk_bias, dv_t, dv_bias, d_rpb, None


def window_attention(qk, qk_bias, v, v_bias, rpb_table, B, H, W, heads, window, shift, scale, C, v_off=0):
    """Swin: qk = v = qkv output [rows,3C], qk_bias = v_bias = qkv.bias, v_off = 2C.
    NeW-CRF: qk = qk output [rows,2C] with its bias; v [rows,C] padded with zeros (v_bias None)."""
    geom = (B, H, W, heads, window, shift, float(scale), C, v_off)
    if v is qk:
        # one tensor feeds q, k and v: pass it once so autograd sums its gradient
        return _WindowAttnFn.apply(qk, qk_bias, qk, qk_bias if v_bias is not None else None, rpb_table, geom)
    return _WindowAttnFn.apply(qk, qk_bias, v, v_bias, rpb_table, geom)


# --------------------------------------------------------------------------
# Adaptive-bin depth head
# --------------------------------------------------------------------------


class _BinHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, centers, do_softmax):
        _require_cuda(logits, centers)
        logits = _c(logits)
        centers = _c(centers)
        B, K = logits.shape[:2]
        HW = logits[0, 0].numel()
        pred = torch.empty(B, 1, *logits.shape[2:], device=logits.device, dtype=torch.float32)
        stats = torch.empty(B, 2, HW, device=logits.device, dtype=torch.float32) if do_softmax else None
        L.call("mdemi_binhead_fwd", logits.data_ptr(), centers.data_ptr(), pred.data_ptr(), L.ptr(stats), None,
               B, K, HW, int(do_softmax), L.stream())
        ctx.save_for_backward(logits, centers, pred, stats)
        ctx.do_softmax = do_softmax
        return pred

    @staticmethod
    def backward(ctx, dpred):
        logits, centers, pred, stats = ctx.saved_tensors
        dpred = _c(dpred)
        B, K = logits.shape[:2]
        HW = logits[0, 0].numel()
        dlogits = torch.empty_like(logits)
        dcenters = torch.empty(B, K, device=logits.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_binhead_bwd_workspace_size(B, K, HW), logits.device)
        L.check(lib.mdemi_binhead_bwd(logits.data_ptr(), centers.data_ptr(), pred.data_ptr(), L.ptr(stats),
                                      dpred.data_ptr(), dlogits.data_ptr(), dcenters.data_ptr(), B, K, HW,
                                      int(ctx.do_softmax), ws.data_ptr(), L.stream()), "binhead_bwd")
        return dlogits, dcenters.view_as(centers), None


def bin_head(logits, centers, do_softmax=True):
    """pred[b,0,...] = sum_k softmax_k(logits)[b,k,...] * centers[b,k]   (NCHW logits)."""
    return _BinHeadFn.apply(logits, centers.reshape(logits.shape[0], logits.shape[1]), do_softmax)


# --------------------------------------------------------------------------
# SILog loss
# --------------------------------------------------------------------------


class _SILogFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, min_depth, alpha, beta, per_image, unbiased):
        _require_cuda(pred, gt)
        pred = _c(pred)
        gt = _c(gt)
        B = pred.shape[0]
        HW = pred[0].numel()
        G = B if per_image else 1
        loss = torch.empty(1, device=pred.device, dtype=torch.float32)
        stats = torch.empty(G, 4, device=pred.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_silog_workspace_size(B, HW), pred.device, slot=2)
        L.check(lib.mdemi_silog_fwd(pred.data_ptr(), gt.data_ptr(), loss.data_ptr(), stats.data_ptr(), B, HW,
                                    float(min_depth), float(alpha), float(beta), int(per_image), int(unbiased),
                                    ws.data_ptr(), L.stream()), "silog_fwd")
        ctx.save_for_backward(pred, gt, stats)
        ctx.cfg = (min_depth, alpha, beta, per_image, unbiased)
        return loss[0]

    @staticmethod
    def backward(ctx, dloss):
        pred, gt, stats = ctx.saved_tensors
        min_depth, alpha, beta, per_image, unbiased = ctx.cfg
        B = pred.shape[0]
        HW = pred[0].numel()
        dpred = torch.empty_like(pred)
        dl = _c(dloss.reshape(1).to(torch.float32))
        L.call("mdemi_silog_bwd", pred.data_ptr(), gt.data_ptr(), stats.data_ptr(), dl.data_ptr(),
               dpred.data_ptr(), B, HW, float(min_depth), float(alpha), float(beta), int(per_image),
               int(unbiased), L.stream())
        return dpred, None, None, None, None, None, None


def silog_loss(pred, gt, min_depth=1e-3, alpha=10.0, beta=0.15, per_image=False, unbiased=False):
    return _SILogFn.apply(pred, gt, min_depth, alpha, beta, per_image, unbiased)


# --------------------------------------------------------------------------
# Resampling / layout
# --------------------------------------------------------------------------


class _BilinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow, align_corners, sh, sw):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, oh, ow, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_bilinear_fwd", x.data_ptr(), y.data_ptr(), n, h, w, c, oh, ow, int(align_corners),
               float(sh), float(sw), c, c, L.stream())
        ctx.cfg = (n, h, w, c, oh, ow, align_corners, sh, sw)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, oh, ow, align_corners, sh, sw = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_bilinear_bwd", dy.data_ptr(), dx.data_ptr(), n, h, w, c, oh, ow, int(align_corners),
               float(sh), float(sw), c, c, 0, L.stream())
        return dx, None, None, None, None, None


def interpolate_bilinear(x_nhwc, size=None, scale_factor=None, align_corners=False):
    n, h, w, c = x_nhwc.shape
    if size is not None:
        oh, ow = size
        sh = sw = 0.0
    else:
        sh = sw = float(scale_factor)
        oh, ow = int(math.floor(h * sh)), int(math.floor(w * sw))
        if align_corners:
            sh = sw = 0.0
    return _BilinearFn.apply(x_nhwc, oh, ow, align_corners, sh, sw)


class _PixelShuffleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, h * r, w * r, c // (r * r), device=x.device, dtype=torch.float32)
        L.call("mdemi_pixel_shuffle_nhwc", x.data_ptr(), y.data_ptr(), n, h, w, c, r, 0, L.stream())
        ctx.cfg = (n, h, w, c, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, r = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_pixel_shuffle_nhwc", dy.data_ptr(), dx.data_ptr(), n, h, w, c, r, 1, L.stream())
        return dx, None


def pixel_shuffle_nhwc(x, r):
    return _PixelShuffleFn.apply(x, r)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, oh, ow, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_adaptive_avgpool_fwd", x.data_ptr(), y.data_ptr(), n, h, w, c, oh, ow, L.stream())
        ctx.cfg = (n, h, w, c, oh, ow)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, oh, ow = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_adaptive_avgpool_bwd", dy.data_ptr(), dx.data_ptr(), n, h, w, c, oh, ow, L.stream())
        return dx, None, None


def adaptive_avg_pool_nhwc(x, out_size):
    oh, ow = (out_size, out_size) if isinstance(out_size, int) else out_size
    return _AvgPoolFn.apply(x, oh, ow)


class _LayoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, to_nhwc):
        _require_cuda(x)
        x = _c(x)
        ctx.to_nhwc = to_nhwc
        if to_nhwc:
            n, c, h, w = x.shape
            y = torch.empty(n, h, w, c, device=x.device, dtype=torch.float32)
            L.call("mdemi_nchw_to_nhwc", x.data_ptr(), y.data_ptr(), n, c, h * w, L.stream())
        else:
            n, h, w, c = x.shape
            y = torch.empty(n, c, h, w, device=x.device, dtype=torch.float32)
            L.call("mdemi_nhwc_to_nchw", x.data_ptr(), y.data_ptr(), n, c, h * w, L.stream())
        return y

    @staticmethod
    def backward(ctx, dy):
        return _LayoutFn.apply(dy, not ctx.to_nhwc), None


def nchw_to_nhwc(x):
    return _LayoutFn.apply(x, True)


def nhwc_to_nchw(x):
    return _LayoutFn.apply(x, False)


# --------------------------------------------------------------------------
# BatchNorm / GroupNorm (training-mode statistics) with fused activation
# --------------------------------------------------------------------------


class _ChNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, groups, is_bn, eps, act, running=None, out_b16=False, pool=False):
        """running: (running_mean, running_var, num_batches_tracked or None, momentum) -- the
        BatchNorm running-statistics update done by the same call (mdemi_bn_train_fwd).
        out_b16: the output feeds a bf16 GEMM -- write its bf16 copy too (bf16 storage).  The
        input gradient gets its bf16 copy when the input came from a conv (its data- and
        weight-gradient GEMMs read it).  pool: the output feeds a SqueezeExcite -- the same
        sweep also writes its per-image spatial mean (mdemi_bn_train_fwd_pooled), recorded on
        the output for squeeze_excite (pooled_of)."""
        _require_cuda(x, weight, bias)
        x = _c(x)
        n = x.shape[0]
        c = x.shape[-1]
        hw = x[0].numel() // c
        y = torch.empty_like(x)
        y16 = new_b16_like(y) if (out_b16 and running is not None and is_bn) else None
        ctx.dx16 = bool(is_bn and grad_feeds_gemm(x))
        nstat = c if is_bn else n * groups
        mean = torch.empty(nstat, device=x.device, dtype=torch.float32)
        rstd = torch.empty(nstat, device=x.device, dtype=torch.float32)
        lib = L.load()
        pool = bool(pool and running is not None and is_bn and c % 4 == 0 and x.data_ptr() % 16 == 0)
        ws = L.workspace(lib.mdemi_bn_train_fwd_pooled_workspace_size(n, hw, c) if pool else
                         lib.mdemi_chnorm_workspace_size(n, hw, c, groups, int(is_bn)), x.device)
        if pool:
            rm, rv, tracked, momentum = running
            pooled = torch.empty(n, c, device=x.device, dtype=torch.float32)
            L.check(lib.mdemi_bn_train_fwd_pooled(x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(),
                                                  L.ptr(y16), pooled.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                                  rm.data_ptr(), rv.data_ptr(), L.ptr(tracked), float(momentum), n,
                                                  hw, c, float(eps), act, ws.data_ptr(), L.stream()),
                    "bn_train_fwd_pooled")
            if y16 is not None:
                set_b16(y, y16)
            y._mdemi_pooled = (pooled, y._version)
        elif running is not None:
            rm, rv, tracked, momentum = running
            L.check(lib.mdemi_bn_train_fwd16(x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(),
                                             L.ptr(y16), mean.data_ptr(), rstd.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                                             L.ptr(tracked), float(momentum), n, hw, c, float(eps), act,
                                             ws.data_ptr(), L.stream()), "bn_train_fwd")
            if y16 is not None:
                set_b16(y, y16)
        else:
            L.check(lib.mdemi_chnorm_fwd(x.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(),
                                         mean.data_ptr(), rstd.data_ptr(), n, hw, c, groups, int(is_bn), float(eps),
                                         act, ws.data_ptr(), L.stream()), "chnorm_fwd")
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.cfg = (groups, is_bn, act)
        ctx.mark_non_differentiable(mean, rstd)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the statistics
        return y, mean, rstd

    @staticmethod
    def backward(ctx, dy, _dm, _dr):
        if dy is None:
            return None, None, None, None, None, None, None, None, None, None
        x, weight, bias, mean, rstd = ctx.saved_tensors
        groups, is_bn, act = ctx.cfg
        dy = _c(dy)
        n = x.shape[0]
        c = x.shape[-1]
        hw = x[0].numel() // c
        dx = torch.empty_like(x)
        dx16 = new_b16_like(dx) if ctx.dx16 else None
        dg = torch.empty(c, device=x.device, dtype=torch.float32)
        db = torch.empty(c, device=x.device, dtype=torch.float32)
        lib = L.load()
        ws = L.workspace(lib.mdemi_chnorm_workspace_size(n, hw, c, groups, int(is_bn)), x.device)
        L.check(lib.mdemi_chnorm_bwd16(dy.data_ptr(), x.data_ptr(), None, mean.data_ptr(), rstd.data_ptr(),
                                       weight.data_ptr(), bias.data_ptr(), dx.data_ptr(), L.ptr(dx16), dg.data_ptr(),
                                       db.data_ptr(), n, hw, c, groups, int(is_bn), act, ws.data_ptr(), L.stream()),
                "chnorm_bwd")
        if dx16 is not None:
            set_b16(dx, dx16)
        return dx, dg, db, None, None, None, None, None, None, None


def batch_norm_nhwc(x, weight, bias, eps=1e-5, act=L.ACT_NONE, running=None, out_b16=False, pool=False):
    """Training-mode BatchNorm2d over an NHWC map; returns (y, batch_mean, batch_rstd).
    running=(running_mean, running_var, num_batches_tracked or None, momentum) also applies
    nn.BatchNorm2d's running-statistics update in the same call.  out_b16: y feeds a bf16
    GEMM (bf16 storage: its bf16 copy is written by the same sweep).  pool: y feeds a
    SqueezeExcite; with running statistics the same sweep records y's per-image spatial mean
    for it (pooled_of)."""
    return _ChNormFn.apply(x, weight, bias, x.shape[-1], True, eps, act, running, out_b16, pool)


def pooled_of(x):
    """The per-image spatial mean [N, C] a BatchNorm sweep recorded on its output x (pool=True),
    if x is unchanged since; else None."""
    rec = x.__dict__.get("_mdemi_pooled")
    if rec is None or rec[1] != x._version or rec[0].shape != (x.shape[0], x.shape[-1]):
        return None
    return rec[0]


def group_norm_nhwc(x, weight, bias, groups, eps=1e-5, act=L.ACT_NONE):
    y, _, _ = _ChNormFn.apply(x, weight, bias, groups, False, eps, act)
    return y


# --------------------------------------------------------------------------
# elementwise
# --------------------------------------------------------------------------


class _SigmoidScaleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        _require_cuda(x)
        x = _c(x)
        y = torch.empty_like(x)
        L.call("mdemi_elementwise", L.EW_SIGMOID_SCALE, x.data_ptr(), None, y.data_ptr(), x.numel(), float(s), 0.0,
               L.stream())
        ctx.save_for_backward(x)
        ctx.s = s
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = _c(dy)
        dx = torch.empty_like(x)
        L.call("mdemi_elementwise", L.EW_SIGMOID_SCALE_BWD, x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(),
               float(ctx.s), 0.0, L.stream())
        return dx, None


def sigmoid_scale(x, s=1.0):
    return _SigmoidScaleFn.apply(x, s)


class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, out_b16):
        _require_cuda(a, b)
        a, b = _c(a), _c(b)
        y = torch.empty_like(a)
        y16 = new_b16_like(y) if (out_b16 and y.numel() % 4 == 0 and a.data_ptr() % 16 == 0
                                  and b.data_ptr() % 16 == 0) else None
        if y16 is not None:
            L.call("mdemi_add16", a.data_ptr(), b.data_ptr(), y.data_ptr(), y16.data_ptr(), a.numel(), L.stream())
            set_b16(y, y16)
        else:
            L.call("mdemi_elementwise", L.EW_ADD, a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), 0.0, 0.0,
                   L.stream())
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy, dy, None


def add(a, b, out_b16=False):
    """a + b; out_b16: the sum feeds a bf16 GEMM (bf16 storage: its bf16 copy in the same sweep)."""
    return _AddFn.apply(a, b, out_b16)


# --------------------------------------------------------------------------
# PatchMerging gather, channel concat, stochastic depth
# --------------------------------------------------------------------------


class _SpaceToDepth2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, (h + 1) // 2, (w + 1) // 2, 4 * c, device=x.device, dtype=torch.float32)
        L.call("mdemi_space_to_depth2", x.data_ptr(), y.data_ptr(), n, h, w, c, 0, L.stream())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c = ctx.shape
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_space_to_depth2", dx.data_ptr(), dy.data_ptr(), n, h, w, c, 1, L.stream())
        return dx


def space_to_depth2(x_nhwc):
    """PatchMerging's x0..x3 gather + cat (swin_transformer.py:272-284), NHWC."""
    return _SpaceToDepth2Fn.apply(x_nhwc)


def _copy2d(src2, dst2, accumulate=False):
    rows, cols = src2.shape
    L.call("mdemi_copy2d", src2.data_ptr(), src2.stride(0), dst2.data_ptr(), dst2.stride(0), rows, cols,
           int(accumulate), L.stream())


class _ConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        _require_cuda(*xs)
        xs = [_c(x) for x in xs]
        lead = xs[0].shape[:-1]
        widths = [x.shape[-1] for x in xs]
        out = torch.empty(*lead, sum(widths), device=xs[0].device, dtype=torch.float32)
        o2 = out.view(-1, out.shape[-1])
        off = 0
        for x, wd in zip(xs, widths):
            _copy2d(x.view(-1, wd), o2[:, off:off + wd])
            off += wd
        ctx.widths = widths
        return out

    @staticmethod
    def backward(ctx, dy):
        dy = _c(dy)
        d2 = dy.view(-1, dy.shape[-1])
        grads = []
        off = 0
        for wd in ctx.widths:
            g = torch.empty(*dy.shape[:-1], wd, device=dy.device, dtype=torch.float32)
            _copy2d(d2[:, off:off + wd], g.view(-1, wd))
            grads.append(g)
            off += wd
        return tuple(grads)


def concat_channels(xs):
    """torch.cat(dim=1) of NCHW maps == channel concat of NHWC maps."""
    return _ConcatFn.apply(*xs)


class _DropPathAddFn(torch.autograd.Function):
    """y = res + branch * scale[sample]  (timm DropPath with scale = keep / (1 - p))."""

    @staticmethod
    def forward(ctx, res, branch, scale):
        res, branch = _c(res), _c(branch)
        y = torch.empty_like(branch)
        per = branch.numel() // scale.numel()
        L.call("mdemi_rowscale_add", res.data_ptr(), branch.data_ptr(), scale.data_ptr(), y.data_ptr(), per,
               branch.numel(), L.stream())
        ctx.save_for_backward(scale)
        ctx.per = per
        return y

    @staticmethod
    def backward(ctx, dy):
        (scale,) = ctx.saved_tensors
        dy = _c(dy)
        db = torch.empty_like(dy)
        L.call("mdemi_rowscale_add", None, dy.data_ptr(), scale.data_ptr(), db.data_ptr(), ctx.per, dy.numel(),
               L.stream())
        return dy, db, None


def drop_path_scale(batch, drop_prob, device):
    """timm DropPath's per-sample scale: bernoulli(keep) / keep, drawn on the device."""
    keep = 1.0 - drop_prob
    return torch.empty(batch, device=device, dtype=torch.float32).bernoulli_(keep).div_(keep)


def drop_path_add(res, branch, drop_prob, training):
    if drop_prob == 0.0 or not training:
        return add(res, branch)
    return _DropPathAddFn.apply(res, branch, drop_path_scale(branch.shape[0], drop_prob, branch.device))


class _BatchNormEvalFn(torch.autograd.Function):
    """BatchNorm2d with running statistics (eval mode), differentiable: a BN frozen by
    freeze_bn (common_utils.py:78-81) inside a training step still passes gradients to
    its input and its affine parameters, as F.batch_norm(training=False) does."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, act):
        _require_cuda(x, weight, bias)
        x = _c(x)
        n, c = x.shape[0], x.shape[-1]
        hw = x[0].numel() // c
        mean = running_mean.detach().clone()  # later running-stat updates must not reach backward
        rstd = torch.rsqrt(running_var.detach() + eps)
        y = torch.empty_like(x)
        L.call("mdemi_chnorm_apply", x.data_ptr(), weight.data_ptr(), bias.data_ptr(), mean.data_ptr(),
               rstd.data_ptr(), y.data_ptr(), n, hw, c, c, 1, act, L.stream())
        ctx.save_for_backward(x, weight, bias, mean, rstd)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, mean, rstd = ctx.saved_tensors
        dy = _c(dy)
        n, c = x.shape[0], x.shape[-1]
        hw = x[0].numel() // c
        want_dx = ctx.needs_input_grad[0]
        want_p = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        dx = torch.empty_like(x) if want_dx else None
        dg = torch.empty(c, device=x.device, dtype=torch.float32) if want_p else None
        db = torch.empty(c, device=x.device, dtype=torch.float32) if want_p else None
        lib = L.load()
        ws = L.workspace(lib.mdemi_chnorm_workspace_size(n, hw, c, c, 1), x.device) if want_p else None
        L.check(lib.mdemi_bn_frozen_bwd(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                        weight.data_ptr(), bias.data_ptr(), L.ptr(dx), L.ptr(dg), L.ptr(db), n, hw, c,
                                        ctx.act, L.ptr(ws), L.stream()), "bn_frozen_bwd")
        return (dx, dg if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None, None, None,
                None, None)


def batch_norm_eval_nhwc(x, weight, bias, running_mean, running_var, eps=1e-5, act=L.ACT_NONE):
    """BatchNorm2d with running statistics over an NHWC map (eval mode); differentiable
    when a gradient is wanted, a single launch otherwise."""
    if torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad or bias.requires_grad):
        return _BatchNormEvalFn.apply(x, weight, bias, running_mean, running_var, eps, act)
    _require_cuda(x)
    x = _c(x)
    n, c = x.shape[0], x.shape[-1]
    hw = x[0].numel() // c
    rstd = torch.rsqrt(running_var + eps)
    y = torch.empty_like(x)
    L.call("mdemi_chnorm_apply", x.data_ptr(), weight.data_ptr(), bias.data_ptr(), running_mean.data_ptr(),
           rstd.data_ptr(), y.data_ptr(), n, hw, c, c, 1, act, L.stream())
    return y


# ==========================================================================
# AdaBins / Depthformer-v8 / EfficientNet-B5 ops (include/mdemi_ext.h)
# ==========================================================================


def _ws(nbytes, device, slot=0):
    return L.workspace(nbytes, device, slot=slot)


class _DWConvFn(torch.autograd.Function):
    """Depthwise KxK conv, NHWC, no bias; pad_t/pad_l + explicit output size (TF 'same')."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad_t, pad_l, oh, ow):
        _require_cuda(x, weight)
        x, weight = _c(x), _c(weight)
        n, h, w, c = x.shape
        k = weight.shape[-1]
        y = torch.empty(n, oh, ow, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_dwconv_fwd", x.data_ptr(), weight.data_ptr(), y.data_ptr(), n, h, w, c, k, stride, pad_t, pad_l,
               oh, ow, L.stream())
        ctx.save_for_backward(x, weight)
        ctx.cfg = (stride, pad_t, pad_l, oh, ow)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, pad_t, pad_l, oh, ow = ctx.cfg
        dy = _c(dy)
        n, h, w, c = x.shape
        k = weight.shape[-1]
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(weight) if ctx.needs_input_grad[1] else None
        lib = L.load()
        ws = _ws(lib.mdemi_dwconv_bwd_workspace_size(n, c, k, oh, ow), x.device)
        L.check(lib.mdemi_dwconv_bwd(dy.data_ptr(), x.data_ptr(), weight.data_ptr(), L.ptr(dx), L.ptr(dw), n, h, w, c,
                                     k, stride, pad_t, pad_l, oh, ow, ws.data_ptr(), L.stream()), "dwconv_bwd")
        return dx, dw, None, None, None, None, None


def same_pad(size, k, s):
    """TF 'same' padding (gen-efficientnet Conv2dSame): output ceil(size/s), extra pad at the end."""
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return out, total // 2


def dwconv_nhwc(x, weight, stride=1, same=True, pad=None):
    n, h, w, c = x.shape
    k = weight.shape[-1]
    if same:
        oh, pt = same_pad(h, k, stride)
        ow, pl = same_pad(w, k, stride)
    else:
        pt = pl = k // 2 if pad is None else pad
        oh = (h + 2 * pt - k) // stride + 1
        ow = (w + 2 * pl - k) // stride + 1
    return _DWConvFn.apply(x, weight, stride, pt, pl, oh, ow)


def spatial_reduce(a, b=None, scale=1.0):
    """out[n, c] = scale * sum_p a[n, p, c] * b[n, p, c]  (NHWC or [N, P, C]); no autograd."""
    n, c = a.shape[0], a.shape[-1]
    hw = a[0].numel() // c
    out = torch.empty(n, c, device=a.device, dtype=torch.float32)
    lib = L.load()
    ws = _ws(lib.mdemi_spatial_reduce_workspace_size(n, hw, c), a.device, slot=3)
    L.check(lib.mdemi_spatial_reduce(a.data_ptr(), L.ptr(b), out.data_ptr(), n, hw, c, float(scale), ws.data_ptr(),
                                     L.stream()), "spatial_reduce")
    return out


def _chan_scale(x, g, add=None, out_b16=False):
    y = torch.empty_like(x)
    n, c = x.shape[0], x.shape[-1]
    y16 = new_b16_like(y) if out_b16 else None
    L.call("mdemi_chan_scale16", x.data_ptr(), g.data_ptr(), L.ptr(add), y.data_ptr(), L.ptr(y16), n,
           x[0].numel() // c, c, L.stream())
    if y16 is not None:
        set_b16(y, y16)
    return y


class _SpatialMeanFn(torch.autograd.Function):
    """mean over the spatial / token axis of an NHWC or [N, P, C] tensor -> [N, C]."""

    @staticmethod
    def forward(ctx, x):
        _require_cuda(x)
        x = _c(x)
        hw = x[0].numel() // x.shape[-1]
        ctx.shape = x.shape
        ctx.hw = hw
        return spatial_reduce(x, None, 1.0 / hw)

    @staticmethod
    def backward(ctx, dy):
        zeros = torch.zeros(ctx.shape, device=dy.device, dtype=torch.float32)
        return _chan_scale(zeros, torch.zeros_like(dy), _scale(_c(dy), 1.0 / ctx.hw))


def spatial_mean(x):
    return _SpatialMeanFn.apply(x)


class _SqueezeExciteFn(torch.autograd.Function):
    """EfficientNet SqueezeExcite: x * sigmoid(W_e swish(W_r mean(x) + b_r) + b_e), NHWC."""

    @staticmethod
    def forward(ctx, x, wr, br, we, be):
        _require_cuda(x, wr, br, we, be)
        x = _c(x)
        n, c = x.shape[0], x.shape[-1]
        hw = x[0].numel() // c
        r = wr.shape[0]
        pooled = pooled_of(x)  # recorded by the BatchNorm sweep that produced x, if it pooled
        if pooled is None:
            pooled = spatial_reduce(x, None, 1.0 / hw)
        hid = torch.empty(n, r, device=x.device, dtype=torch.float32)
        gate = torch.empty(n, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_se_gate_fwd", pooled.data_ptr(), _c(wr).data_ptr(), br.data_ptr(), _c(we).data_ptr(),
               be.data_ptr(), hid.data_ptr(), gate.data_ptr(), n, c, r, L.stream())
        y = _chan_scale(x, gate, out_b16=True)  # SqueezeExcite's output feeds the projection conv
        ctx.save_for_backward(x, wr, we, pooled, hid, gate)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wr, we, pooled, hid, gate = ctx.saved_tensors
        dy = _c(dy)
        n, c = x.shape[0], x.shape[-1]
        hw = x[0].numel() // c
        r = wr.shape[0]
        dgate = spatial_reduce(dy, x, 1.0)
        dpooled = torch.empty(n, c, device=x.device, dtype=torch.float32)
        dwr, dbr = torch.empty_like(wr), torch.empty(r, device=x.device, dtype=torch.float32)
        dwe, dbe = torch.empty_like(we), torch.empty(c, device=x.device, dtype=torch.float32)
        lib = L.load()
        ws = _ws(lib.mdemi_se_gate_bwd_workspace_size(n, c, r), x.device, slot=3)
        L.check(lib.mdemi_se_gate_bwd(pooled.data_ptr(), _c(wr).data_ptr(), _c(we).data_ptr(), hid.data_ptr(),
                                      gate.data_ptr(), dgate.data_ptr(), dpooled.data_ptr(), dwr.data_ptr(),
                                      dbr.data_ptr(), dwe.data_ptr(), dbe.data_ptr(), n, c, r, 1.0 / hw,
                                      ws.data_ptr(), L.stream()), "se_gate_bwd")
        # d/dx of x * gate plus the pooling path: dpooled / HW (scaled by se_gate_bwd) broadcast
        dx = _chan_scale(dy, gate, dpooled)
        return dx, dwr, dbr, dwe, dbe


def _scale(t, s):
    out = torch.empty_like(t)
    L.call("mdemi_elementwise", L.EW_AXPBY, t.data_ptr(), t.data_ptr(), out.data_ptr(), t.numel(), float(s), 0.0,
           L.stream())
    return out


def squeeze_excite(x, wr, br, we, be):
    """wr [R, C], we [C, R] (the 1x1 conv weights flattened)."""
    return _SqueezeExciteFn.apply(x, wr, br, we, be)


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale):
        _require_cuda(x)
        x = _c(x)
        cols = x.shape[-1]
        y = torch.empty_like(x)
        L.call("mdemi_softmax_fwd", x.data_ptr(), y.data_ptr(), x.numel() // cols, cols, float(scale), L.stream())
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = _c(dy)
        cols = y.shape[-1]
        dx = torch.empty_like(y)
        L.call("mdemi_softmax_bwd", y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel() // cols, cols,
               float(ctx.scale), 0, L.stream())
        return dx, None


def softmax_lastdim(x, scale=1.0):
    """softmax(scale * x, dim=-1)."""
    return _SoftmaxFn.apply(x, scale)


_drop_counter = [0]


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        _require_cuda(x)
        x = _c(x)
        y = torch.empty_like(x)
        _drop(x.data_ptr(), y.data_ptr(), x.numel(), p, seed, offset=offset)
        ctx.cfg = (p, seed, offset)
        ctx.dx16 = grad_feeds_gemm(x) and x.numel() % 4 == 0
        return y

    @staticmethod
    def backward(ctx, dy):
        p, seed, offset = ctx.cfg
        dy = _c(dy)
        dx = torch.empty_like(dy)
        dx16 = new_b16_like(dx) if ctx.dx16 and dy.data_ptr() % 16 == 0 else None
        _drop(dy.data_ptr(), dx.data_ptr(), dy.numel(), p, seed, offset=offset, dst16_ptr=L.ptr(dx16))
        if dx16 is not None:
            set_b16(dx, dx16)
        return dx, None, None, None


def dropout(x, p, training):
    """Inverted dropout; the mask is a hash of (seed, element index) with the seed drawn on the
    GPU once per call, so the backward regenerates it instead of storing it."""
    if not training or p == 0.0:
        return x
    seed = _draw_seed(x.device)
    off = _drop_counter[0]
    _drop_counter[0] += x.numel()
    return _DropoutFn.apply(x, p, seed, off)


class _BinHeadNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, centers):
        _require_cuda(logits, centers)
        logits, centers = _c(logits), _c(centers)
        b, k = logits.shape[0], logits.shape[-1]
        hw = logits[0].numel() // k
        pred = torch.empty(b, hw, device=logits.device, dtype=torch.float32)
        stats = torch.empty(b, hw, 2, device=logits.device, dtype=torch.float32)
        L.call("mdemi_binhead_nhwc_fwd", logits.data_ptr(), centers.data_ptr(), pred.data_ptr(), stats.data_ptr(), b,
               hw, k, L.stream())
        ctx.save_for_backward(logits, centers, pred, stats)
        return pred

    @staticmethod
    def backward(ctx, dpred):
        logits, centers, pred, stats = ctx.saved_tensors
        dpred = _c(dpred)
        b, k = logits.shape[0], logits.shape[-1]
        hw = logits[0].numel() // k
        dlogits = torch.empty_like(logits)
        dcenters = torch.empty(b, k, device=logits.device, dtype=torch.float32)
        lib = L.load()
        ws = _ws(lib.mdemi_binhead_nhwc_bwd_workspace_size(b, hw, k), logits.device)
        L.check(lib.mdemi_binhead_nhwc_bwd(logits.data_ptr(), centers.data_ptr(), pred.data_ptr(), stats.data_ptr(),
                                           dpred.data_ptr(), dlogits.data_ptr(), dcenters.data_ptr(), b, hw, k,
                                           ws.data_ptr(), L.stream()), "binhead_nhwc_bwd")
        return dlogits, dcenters.view_as(centers)


def bin_head_nhwc(logits, centers):
    """logits [B, H, W, K] (channels-last) -> pred [B, 1, H, W] = sum_k softmax(logits)_k * centers[b, k]."""
    b, h, w, k = logits.shape
    return _BinHeadNHWCFn.apply(logits, centers.reshape(b, k)).view(b, 1, h, w)


class _BinsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, mode, min_val, max_val):
        _require_cuda(raw)
        raw = _c(raw)
        b, k = raw.shape
        widths = torch.empty(b, k, device=raw.device, dtype=torch.float32)
        edges = torch.empty(b, k + 1, device=raw.device, dtype=torch.float32)
        centers = torch.empty(b, k, device=raw.device, dtype=torch.float32)
        L.call("mdemi_bins_fwd", raw.data_ptr(), widths.data_ptr(), edges.data_ptr(), centers.data_ptr(), b, k,
               mode, float(min_val), float(max_val), L.stream())
        ctx.save_for_backward(raw)
        ctx.cfg = (mode, min_val, max_val)
        ctx.set_materialize_grads(False)
        return widths, edges, centers

    @staticmethod
    def backward(ctx, dwidths, dedges, dcenters):
        (raw,) = ctx.saved_tensors
        mode, min_val, max_val = ctx.cfg
        b, k = raw.shape
        dc = _c(dcenters) if dcenters is not None else torch.zeros(b, k, device=raw.device, dtype=torch.float32)
        draw = torch.empty_like(raw)
        L.call("mdemi_bins_bwd", raw.data_ptr(), dc.data_ptr(), L.ptr(_c(dedges) if dedges is not None else None),
               L.ptr(_c(dwidths) if dwidths is not None else None), draw.data_ptr(), b, k, mode, float(min_val),
               float(max_val), L.stream())
        return draw, None, None, None


def bins_from_raw(raw, mode, min_val, max_val, with_widths=False):
    """Regressor output [B, K] -> (bin_edges [B, K+1], centers [B, K]) (and the normalised widths
    first when with_widths).  mode: L.BINS_RELU (AdaBins norm='linear') or L.BINS_ELU
    (Depthformer v8)."""
    w, e, c = _BinsFn.apply(raw, mode, min_val, max_val)
    return (w, e, c) if with_widths else (e, c)


def nchw_to_nhwc_pad(x, cp):
    """Image NCHW -> NHWC with channels zero-padded to cp (no autograd: the image is an input)."""
    _require_cuda(x)
    x = _c(x)
    n, c, h, w = x.shape
    y = torch.empty(n, h, w, cp, device=x.device, dtype=torch.float32)
    L.call("mdemi_nchw_to_nhwc_pad", x.data_ptr(), y.data_ptr(), n, c, h * w, cp, L.stream())
    return y


def depth_metrics(pred, gt, rect, min_depth, max_depth, clamp_pred=True):
    """Per-image [a1, a2, a3, abs_rel, sq_rel, rmse, rmse_log, silog, log_10, n_valid] (fp64) over
    crop rect (y0, y1, x0, x1) & min_depth < gt < max_depth (utils/depth_utils.py:4-54)."""
    _require_cuda(pred, gt)
    pred, gt = _c(pred), _c(gt)
    b = pred.shape[0]
    h, w = pred.shape[-2:]
    out = torch.empty(b, 10, device=pred.device, dtype=torch.float64)
    lib = L.load()
    ws = _ws(lib.mdemi_depth_metrics_workspace_size(b, h, w), pred.device, slot=3)
    y0, y1, x0, x1 = rect
    L.check(lib.mdemi_depth_metrics(pred.data_ptr(), gt.data_ptr(), b, h, w, y0, y1, x0, x1, float(min_depth),
                                    float(max_depth), int(clamp_pred), out.data_ptr(), ws.data_ptr(), L.stream()),
            "depth_metrics")
    return out


def conv_weight_layout(w, mode, conv_shape=None):
    """Conv weight re-layout on the GPU (mdemi_conv_weight_layout): L.WL_OHWI / L.WL_DGRAD take
    the reference's [Cout][Cin][KH][KW] weight; L.WL_OIHW takes [Cout][KH][KW][Cin] data and
    returns the parameter layout (conv_shape = (Cout, Cin, KH, KW) names the conv).  1x1
    OHWI/OIHW re-layouts are identities and return a view."""
    cout, cin, kh, kw = conv_shape if conv_shape is not None else w.shape
    w = _c(w)
    if kh == 1 and kw == 1 and mode != L.WL_DGRAD:
        return w.view(cout, cin, 1, 1) if mode == L.WL_OIHW else w.view(cout, 1, 1, cin)
    shape = {L.WL_OHWI: (cout, kh, kw, cin), L.WL_OIHW: (cout, cin, kh, kw), L.WL_DGRAD: (kh, kw, cout, cin)}[mode]
    out = torch.empty(shape, device=w.device, dtype=torch.float32)
    # a GEMM operand (forward / input-gradient layouts) under bf16 storage: its bf16 copy in the
    # same sweep, instead of a cast of the fresh re-laid-out weight by the GEMM
    out16 = new_b16_like(out) if mode != L.WL_OIHW else None
    L.call("mdemi_conv_weight_layout16", w.data_ptr(), out.data_ptr(), L.ptr(out16), cout, cin, kh, kw, mode,
           L.stream())
    if out16 is not None:
        set_b16(out, out16)
    return out


def flip_w(x):
    """x flipped along its last (width) dim, e.g. an NCHW image batch for flip-eval."""
    _require_cuda(x)
    x = _c(x)
    y = torch.empty_like(x)
    if x.numel():
        w = x.shape[-1]
        L.call("mdemi_flip_w", x.data_ptr(), y.data_ptr(), x.numel() // w, w, L.stream())
    return y


def flip_avg_w(a, b):
    """(a + b flipped along width) / 2: the flip-eval average of a prediction and the
    prediction of the flipped input."""
    _require_cuda(a, b)
    if a.shape != b.shape:
        raise ValueError(f"flip_avg_w: shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    a, b = _c(a), _c(b)
    y = torch.empty_like(a)
    if a.numel():
        w = a.shape[-1]
        L.call("mdemi_flip_avg_w", a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel() // w, w, L.stream())
    return y


class _BinsChamferFn(torch.autograd.Function):
    """Bin-centre chamfer loss (upstream AdaBins BinsChamferLoss over pytorch3d chamfer_distance
    defaults; the reference's loss module is absent -- parity unpinned): batch mean of
    cham_x (centre -> nearest valid GT depth) + cham_y (valid GT depth -> nearest centre).
    The forward also writes dloss/dcentres, so the backward is one sweep onto the input."""

    @staticmethod
    def forward(ctx, bins, gt, thresh, from_edges):
        _require_cuda(bins, gt)
        shape = bins.shape
        bins, gt = _c(bins.reshape(shape[0], -1)), _c(gt)
        B, n = bins.shape
        if gt.shape[0] != B:
            raise ValueError(f"bins_chamfer: batch mismatch {B} vs {gt.shape[0]}")
        fe = 1 if from_edges else 0
        P, HW = n - fe, gt.numel() // B
        if P < 1 or HW < 1:
            raise ValueError(f"bins_chamfer: empty bins {tuple(shape)} or targets {tuple(gt.shape)}")
        loss = torch.empty((), device=bins.device, dtype=torch.float32)
        gcent = torch.empty(B, P, device=bins.device, dtype=torch.float32)
        lib = L.load()
        ws = _ws(lib.mdemi_bins_chamfer_workspace_size(B, P, HW), bins.device, slot=3)
        L.check(lib.mdemi_bins_chamfer_fwd(bins.data_ptr(), gt.data_ptr(), B, P, fe, HW, float(thresh),
                                           loss.data_ptr(), gcent.data_ptr(), ws.data_ptr(), L.stream()),
                "bins_chamfer_fwd")
        ctx.save_for_backward(gcent)
        ctx.cfg = (fe, shape)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        (gcent,) = ctx.saved_tensors
        fe, shape = ctx.cfg
        B, P = gcent.shape
        dloss = _c(dloss.reshape(1).float())
        dbins = torch.empty(B, P + fe, device=gcent.device, dtype=torch.float32)
        L.call("mdemi_bins_chamfer_bwd", gcent.data_ptr(), dloss.data_ptr(), dbins.data_ptr(), B, P, fe, L.stream())
        return dbins.view(shape), None, None, None


def bins_chamfer(bins, gt, thresh=1e-3, from_edges=True):
    """Chamfer loss between each image's bin centres and its GT depths >= thresh, batch-averaged.
    bins: bin edges (B, P+1) (AdaBins; centres are edge midpoints) or, with from_edges=False,
    the centres themselves (B, P, ...) (Depthformer v8); gt (B, 1, H, W)."""
    return _BinsChamferFn.apply(bins, gt, thresh, from_edges)


class _AttentionFn(torch.autograd.Function):
    """Multi-head scaled dot-product attention over column slices of token-major buffers
    ([B*S, ld] rows): per head h, P = softmax(scale * Q_h K_h^T) (returned, [B, heads, Sq, Sk]),
    O_h = dropout(P) V_h written to out[:, h*dv:(h+1)*dv].  QK^T / PV / their gradients are
    batched MFMA GEMMs (batch = B); softmax and dropout are row sweeps.  Serves
    nn.TransformerEncoderLayer's self-attention (layers.py:8), PreNormLunaBlock's two
    attentions (luna_layer.py:202-250) and SelfAttentionBlock (self_attention.py:61-80)."""

    @staticmethod
    def forward(ctx, qsrc, ksrc, vsrc, cfg, out_b16=False):
        B, Sq, Sk, heads, dqk, dv, q_off, k_off, v_off, scale, p, seed = cfg
        _require_cuda(qsrc, ksrc, vsrc)
        ldq, ldk, ldv = qsrc.shape[-1], ksrc.shape[-1], vsrc.shape[-1]
        dev = qsrc.device
        P = torch.empty(B, heads, Sq, Sk, device=dev, dtype=torch.float32)
        hs = Sq * Sk
        gemm(qsrc, ksrc, P, Sq, Sk, dqk, lda=ldq, ldb=ldk, ldc=Sk, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
             batch=B * heads, a_bstride=Sq * ldq, b_bstride=Sk * ldk, c_bstride=heads * hs, a_off=q_off,
             b_off=k_off, inner=(heads, dqk, dqk, hs))
        # bf16 storage: the probabilities' bf16 copy (P.V's operand) from the softmax sweep, or the
        # dropped-out ones' from the dropout sweep
        P16 = new_b16_like(P) if (p == 0.0 or P.numel() % 4 == 0) else None
        out = torch.empty(B * Sq, heads * dv, device=dev, dtype=torch.float32)
        out16 = new_b16_like(out) if out_b16 else None  # the output projection's operand
        pv = dict(lda=Sk, ldb=ldv, ldc=heads * dv, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG, batch=B * heads,
                  a_bstride=heads * hs, b_bstride=Sk * ldv, c_bstride=Sq * heads * dv, b_off=v_off,
                  inner=(heads, hs, dv, dv), c16=out16)
        ctx.P16d = None
        v16 = b16_of(vsrc) if (p > 0.0 and P16 is not None and _FUSE_DROP[0]) else None
        softmaxed = False  # P holds softmax(scale * P) already (the sweep runs in place: never twice)
        if v16 is not None:
            # fused attention dropout (bf16 storage): the softmax sweep writes P and the bf16 copy of
            # dropout(P), P.V reads that copy; no dropout sweep, no fp32 dropout(P)
            L.call("mdemi_softmax_fwd_drop16", P.data_ptr(), P.data_ptr(), P16.data_ptr(), B * heads * Sq, Sk,
                   float(scale), float(p), seed.data_ptr(), 0, 0, L.stream())
            softmaxed = True
            try:
                gemm(None, vsrc, out, Sq, dv, Sk, a16=P16, b16=v16, **pv)
                ctx.P16d = P16  # dropout(P) in bf16: dV's operand in the backward
            except B16Unsupported:  # V's bf16 slice cannot be staged: the fp32 dropout(P) below
                v16 = None
        if v16 is None:
            if not softmaxed:
                L.call("mdemi_softmax_fwd16", P.data_ptr(), P.data_ptr(), L.ptr(P16) if p == 0.0 else None,
                       B * heads * Sq, Sk, float(scale), L.stream())
            Pd = P
            if p > 0.0:
                Pd = torch.empty_like(P)
                _drop(P.data_ptr(), Pd.data_ptr(), P.numel(), p, seed, dst16_ptr=L.ptr(P16))
            if P16 is not None:
                set_b16(Pd, P16)
            gemm(Pd, vsrc, out, Sq, dv, Sk, **pv)
        if out16 is not None:
            set_b16(out, out16)
        ctx.save_for_backward(qsrc, ksrc, vsrc, P)
        ctx.cfg = cfg
        ctx.grad16 = tuple(grad_feeds_gemm(t) for t in (qsrc, ksrc, vsrc))
        ctx.set_materialize_grads(False)  # unused probabilities: no zero fill + add of [B,h,Sq,Sk]
        return out, P

    @staticmethod
    def backward(ctx, dout, dP_ext):
        qsrc, ksrc, vsrc, P = ctx.saved_tensors
        B, Sq, Sk, heads, dqk, dv, q_off, k_off, v_off, scale, p, seed = ctx.cfg
        ldq, ldk, ldv = qsrc.shape[-1], ksrc.shape[-1], vsrc.shape[-1]
        hs = Sq * Sk
        Pd, Pd16 = P, None
        if p > 0.0 and ctx.P16d is not None:
            Pd, Pd16 = None, ctx.P16d  # the forward's bf16 dropout(P): dV's operand, no regeneration
        elif p > 0.0:
            Pd = torch.empty_like(P)
            _drop(P.data_ptr(), Pd.data_ptr(), P.numel(), p, seed)
        ctx.P16d = None
        # one gradient buffer per distinct source tensor; columns outside the used slices are zero
        bufs, spans, b16s = {}, {}, {}
        for t, off, width in ((qsrc, q_off, heads * dqk), (ksrc, k_off, heads * dqk), (vsrc, v_off, heads * dv)):
            spans.setdefault(id(t), []).append((off, width))
        want16 = {}
        for t, w in zip((qsrc, ksrc, vsrc), ctx.grad16):
            want16[id(t)] = want16.get(id(t), False) or w
        for t in (qsrc, ksrc, vsrc):
            if id(t) in bufs:
                continue
            covered = sum(w for _, w in spans[id(t)])
            full = covered == t.shape[-1] and dout is not None
            bufs[id(t)] = torch.empty_like(t) if full else torch.zeros_like(t)
            # a fully written gradient that a GEMM backward reads next: its bf16 copy too
            b16s[id(t)] = new_b16_like(t) if full and want16[id(t)] else None
        dq, dk, dvv = bufs[id(qsrc)], bufs[id(ksrc)], bufs[id(vsrc)]
        dq16, dk16, dv16 = b16s[id(qsrc)], b16s[id(ksrc)], b16s[id(vsrc)]
        dP = torch.empty_like(P)
        if dout is not None:
            dout = _c(dout)
            gemm(dout, vsrc, dP, Sq, Sk, dv, lda=heads * dv, ldb=ldv, ldc=Sk, a_layout=L.L_KCONTIG,
                 b_layout=L.L_KCONTIG, batch=B * heads, a_bstride=Sq * heads * dv, b_bstride=Sk * ldv,
                 c_bstride=heads * hs, b_off=v_off, inner=(heads, dv, dv, hs))
            dvk = dict(lda=Sk, ldb=heads * dv, ldc=ldv, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                       batch=B * heads, a_bstride=heads * hs, b_bstride=Sq * heads * dv, c_bstride=Sk * ldv,
                       c_off=v_off, inner=(heads, hs, dv, dv), c16=dv16)
            o16 = b16_of(dout) if Pd16 is not None else None
            try:
                if o16 is None and Pd16 is not None:
                    raise B16Unsupported("dO has no bf16 copy")
                gemm(Pd, dout, dvv, Sk, dv, Sq, a16=Pd16, b16=o16, **dvk)
            except B16Unsupported:  # regenerate dropout(P) in fp32 instead
                Pd = torch.empty_like(P)
                _drop(P.data_ptr(), Pd.data_ptr(), P.numel(), p, seed)
                gemm(Pd, dout, dvv, Sk, dv, Sq, **dvk)
            if p > 0.0:
                _drop(dP.data_ptr(), dP.data_ptr(), dP.numel(), p, seed)
            if dP_ext is not None:
                dP_ext = _c(dP_ext)
                L.call("mdemi_elementwise", L.EW_ADD, dP.data_ptr(), dP_ext.data_ptr(), dP.data_ptr(), dP.numel(),
                       0.0, 0.0, L.stream())
        elif dP_ext is not None:  # only the returned probabilities carry a gradient
            _copy2d(_c(dP_ext).view(-1, Sk), dP.view(-1, Sk))
        else:
            dP.zero_()
        dP16 = new_b16_like(dP)  # dS: the operand of the dQ and dK GEMMs
        L.call("mdemi_softmax_bwd16", P.data_ptr(), dP.data_ptr(), dP.data_ptr(), L.ptr(dP16), B * heads * Sq, Sk,
               float(scale), 0, L.stream())
        if dP16 is not None:
            set_b16(dP, dP16)
        gemm(dP, ksrc, dq, Sq, dqk, Sk, lda=Sk, ldb=ldk, ldc=ldq, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG,
             batch=B * heads, a_bstride=heads * hs, b_bstride=Sk * ldk, c_bstride=Sq * ldq, b_off=k_off,
             c_off=q_off, inner=(heads, hs, dqk, dqk), c16=dq16)
        gemm(dP, qsrc, dk, Sk, dqk, Sq, lda=Sk, ldb=ldq, ldc=ldk, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             batch=B * heads, a_bstride=heads * hs, b_bstride=Sq * ldq, c_bstride=Sk * ldk, b_off=q_off,
             c_off=k_off, inner=(heads, hs, dqk, dqk), c16=dk16)
        for t in (qsrc, ksrc, vsrc):
            if b16s[id(t)] is not None:
                set_b16(bufs[id(t)], b16s[id(t)])
        seen, grads = set(), []
        for t, g in ((qsrc, dq), (ksrc, dk), (vsrc, dvv)):
            grads.append(None if id(t) in seen else g)
            seen.add(id(t))
        return grads[0], grads[1], grads[2], None, None


def attention(qsrc, ksrc, vsrc, B, Sq, Sk, heads, dqk, dv, scale, q_off=0, k_off=0, v_off=0, p=0.0,
              training=False, out_b16=False):
    """Returns (out [B*Sq, heads*dv], probs [B, heads, Sq, Sk]).  q/k/v are column slices
    (offsets q_off/k_off/v_off, head-major) of 2-D token-major buffers [B*S, ld]; a buffer may
    feed several of them (e.g. a fused qkv projection).  out_b16: `out` feeds a bf16 GEMM
    (the output projection) -- write its bf16 copy too (bf16 storage)."""
    p = float(p) if training else 0.0
    seed = _draw_seed(qsrc.device) if p > 0.0 else None
    cfg = (B, Sq, Sk, heads, dqk, dv, q_off, k_off, v_off, float(scale), p, seed)
    return _AttentionFn.apply(_c(qsrc), _c(ksrc), _c(vsrc), cfg, out_b16)


def _bgemm_raw(A, B, ta, tb, bias=None):
    """C[b] = op(A[b]) @ op(B[b]) (+ bias[j]); A/B dense [nb, r, c] or [r, c] / [1, r, c] (shared)."""
    nb = max(A.shape[0] if A.dim() == 3 else 1, B.shape[0] if B.dim() == 3 else 1)
    ar, ac = A.shape[-2:]
    br, bc = B.shape[-2:]
    M, K = (ac, ar) if ta else (ar, ac)
    K2, N = (bc, br) if tb else (br, bc)
    if K != K2:
        raise ValueError(f"bgemm: inner sizes differ ({K} vs {K2})")
    C = torch.empty(nb, M, N, device=A.device, dtype=torch.float32)
    a_bs = ar * ac if (A.dim() == 3 and A.shape[0] > 1) else 0
    b_bs = br * bc if (B.dim() == 3 and B.shape[0] > 1) else 0
    gemm(A, B, C, M, N, K, lda=ac, ldb=bc, ldc=N, a_layout=L.L_MNCONTIG if ta else L.L_KCONTIG,
         b_layout=L.L_KCONTIG if tb else L.L_MNCONTIG, batch=nb, a_bstride=a_bs, b_bstride=b_bs,
         c_bstride=M * N, bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE)
    return C


class _BatchedGemmFn(torch.autograd.Function):
    """C[b] = op(A[b]) @ op(B[b]) (+ bias[j]), op = transpose when flagged; A or B may be shared
    by every batch entry (stored once).  Serves PixelWiseDotProduct (layers.py:38-43) and the
    conv_out-folded bin logits of AdaBins (unet_adaptive_bins.py:88-97)."""

    @staticmethod
    def forward(ctx, A, B, bias, ta, tb):
        _require_cuda(A, B, bias)
        A, B = _c(A), _c(B)
        C = _bgemm_raw(A, B, ta, tb, bias)
        ctx.save_for_backward(A, B)
        shared_a = not (A.dim() == 3 and A.shape[0] > 1)
        shared_b = not (B.dim() == 3 and B.shape[0] > 1)
        ctx.cfg = (ta, tb, C.shape[0], shared_a, shared_b, bias is not None)
        return C

    @staticmethod
    def backward(ctx, dC):
        A, B = ctx.saved_tensors
        ta, tb, nb, shared_a, shared_b, has_bias = ctx.cfg
        dC = _c(dC)

        def run(X, tx, Y, ty, shared):
            out = _bgemm_raw(X, Y, tx, ty)
            if shared and nb > 1:  # sum the per-entry gradients of a shared operand
                red = torch.empty(out.shape[1:], device=out.device, dtype=torch.float32)
                colsum(out.view(nb, -1), out=red.view(-1))
                return red
            return out

        dA = dB = db = None
        if ctx.needs_input_grad[0]:
            # not ta: dA = dC op(B)^T ; ta: dA = op(B) dC^T
            dA = run(dC, False, B, not tb, shared_a) if not ta else run(B, tb, dC, True, shared_a)
            dA = dA.view_as(A)
        if ctx.needs_input_grad[1]:
            # not tb: dB = op(A)^T dC ; tb: dB = dC^T op(A)
            dB = run(A, not ta, dC, False, shared_b) if not tb else run(dC, True, A, ta, shared_b)
            dB = dB.view_as(B)
        if has_bias and ctx.needs_input_grad[2]:
            db = colsum(dC.view(-1, dC.shape[-1]))
        return dA, dB, db, None, None


def bgemm(A, B, bias=None, ta=False, tb=False):
    """Batched op(A) @ op(B) on MFMA tiles; A/B are [nb, r, c] or [r, c] (shared over the batch)."""
    return _BatchedGemmFn.apply(A, B, bias, ta, tb)


class _UpConcatFn(torch.autograd.Function):
    """cat([resize(x), skip], channels) (unet_adaptive_bins.py:22-23) or cat([skip, resize(x)])
    (layer_utils.py:114-120): the bilinear sweep writes straight into its channel slice."""

    @staticmethod
    def forward(ctx, x, skip, oh, ow, align, sh, sw, x_first):
        _require_cuda(x, skip)
        x, skip = _c(x), _c(skip)
        n, h, w, cx = x.shape
        cs = skip.shape[-1]
        out = torch.empty(n, oh, ow, cx + cs, device=x.device, dtype=torch.float32)
        ct = cx + cs
        xo, so = (0, cx) if x_first else (cs, 0)
        L.call("mdemi_bilinear_fwd", x.data_ptr(), out.data_ptr() + 4 * xo, n, h, w, cx, oh, ow, int(align), float(sh),
               float(sw), cx, ct, L.stream())
        _copy2d(skip.view(-1, cs), out.view(-1, ct)[:, so:so + cs])
        ctx.cfg = (n, h, w, cx, cs, oh, ow, align, sh, sw, xo, so)
        return out

    @staticmethod
    def backward(ctx, dy):
        n, h, w, cx, cs, oh, ow, align, sh, sw, xo, so = ctx.cfg
        dy = _c(dy)
        ct = cx + cs
        dx = torch.empty(n, h, w, cx, device=dy.device, dtype=torch.float32)
        L.call("mdemi_bilinear_bwd", dy.data_ptr() + 4 * xo, dx.data_ptr(), n, h, w, cx, oh, ow, int(align), float(sh),
               float(sw), ct, cx, 0, L.stream())
        ds = torch.empty(n, oh, ow, cs, device=dy.device, dtype=torch.float32)
        _copy2d(dy.view(-1, ct)[:, so:so + cs], ds.view(-1, cs))
        return dx, ds, None, None, None, None, None, None


def upsample_concat(x, skip, size=None, scale_factor=None, align_corners=True, x_first=True):
    n, h, w, c = x.shape
    if size is not None:
        oh, ow = size
        sh = sw = 0.0
    else:
        oh, ow = int(math.floor(h * scale_factor)), int(math.floor(w * scale_factor))
        sh = sw = 0.0 if align_corners else float(scale_factor)
    return _UpConcatFn.apply(x, skip, oh, ow, align_corners, sh, sw, x_first)


class _LinearActFn(torch.autograd.Function):
    """act(x W^T + b) with the activation in the GEMM epilogue (pre-activation kept for the
    backward): nn.Sequential(Linear, LeakyReLU/SiLU) stacks (miniViT.py:19-23,
    decoder_v8.py:82-90)."""

    @staticmethod
    def forward(ctx, x, weight, bias, act):
        _require_cuda(x, weight, bias)
        K = x.shape[-1]
        x2 = _c(x).reshape(-1, K)
        M, N = x2.shape[0], weight.shape[0]
        out = torch.empty(M, N, device=x.device, dtype=torch.float32)
        pre = torch.empty(M, N, device=x.device, dtype=torch.float32)
        gemm(x2, _c(weight), out, M, N, K, lda=K, ldb=K, ldc=N, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
             bias=bias, bias_mode=L.BIAS_COL if bias is not None else L.BIAS_NONE, act=act, preact=pre, ldpre=N,
             split_k=1)
        ctx.save_for_backward(x2, weight, pre)
        ctx.act = act
        ctx.has_bias = bias is not None
        ctx.xshape = x.shape
        return out.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, pre = ctx.saved_tensors
        dy2 = _c(dy).reshape(pre.shape)
        dpre = torch.empty_like(pre)
        L.call("mdemi_elementwise", L.EW_ACT_BWD, pre.data_ptr(), dy2.data_ptr(), dpre.data_ptr(), pre.numel(),
               float(ctx.act), 0.0, L.stream())
        M, K = x2.shape
        N = weight.shape[0]
        dx = torch.empty(M, K, device=dy.device, dtype=torch.float32)
        gemm(dpre, weight, dx, M, K, N, lda=N, ldb=K, ldc=K, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG)
        dw = torch.empty(N, K, device=dy.device, dtype=torch.float32)
        db = torch.empty(N, device=dy.device, dtype=torch.float32) if ctx.has_bias else None
        gemm(dpre, x2, dw, N, K, M, lda=N, ldb=K, ldc=K, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG, rowsum_a=db)
        return dx.view(ctx.xshape), dw, db, None


def linear_act(x, weight, bias, act):
    return _LinearActFn.apply(x, weight, bias, act)


class _RowsFn(torch.autograd.Function):
    """x[b, start:start+count, :] for every b of a [B, S, C] tensor, as a dense [B, count, C]."""

    @staticmethod
    def forward(ctx, x, start, count):
        _require_cuda(x)
        x = _c(x)
        B, S, C = x.shape
        out = torch.empty(B, count, C, device=x.device, dtype=torch.float32)
        src = x.view(B, S * C)[:, start * C:(start + count) * C]
        _copy2d(src, out.view(B, count * C))
        ctx.cfg = (B, S, C, start, count)
        return out

    @staticmethod
    def backward(ctx, dy):
        B, S, C, start, count = ctx.cfg
        dx = torch.zeros(B, S, C, device=dy.device, dtype=torch.float32)
        _copy2d(_c(dy).view(B, count * C), dx.view(B, S * C)[:, start * C:(start + count) * C])
        return dx, None, None


def take_rows(x, start, count):
    return _RowsFn.apply(x, start, count)


class _AddRowsBroadcastFn(torch.autograd.Function):
    """y[b] = x[b] + t[:S] for x [B, S, C]: the learned positional encodings (layers.py:26)."""

    @staticmethod
    def forward(ctx, x, table):
        _require_cuda(x, table)
        x = _c(x)
        B, S, C = x.shape
        y = torch.empty_like(x)
        _copy2d(x.view(B, S * C), y.view(B, S * C))
        L.call("mdemi_copy2d", _c(table).data_ptr(), 0, y.data_ptr(), S * C, B, S * C, 1, L.stream())
        ctx.cfg = (B, S, C, table.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        B, S, C, tshape = ctx.cfg
        dy = _c(dy)
        dt = torch.zeros(tshape, device=dy.device, dtype=torch.float32)
        colsum(dy.view(B, S * C), out=dt.view(-1)[:S * C])
        return dy, dt


def add_rows_broadcast(x, table):
    return _AddRowsBroadcastFn.apply(x, table)


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        _require_cuda(x)
        x = _c(x)
        y = torch.empty_like(x)
        L.call("mdemi_act_fwd", x.data_ptr(), y.data_ptr(), x.numel(), act, L.stream())
        ctx.save_for_backward(x)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = _c(dy)
        dx = torch.empty_like(x)
        L.call("mdemi_elementwise", L.EW_ACT_BWD, x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(),
               float(ctx.act), 0.0, L.stream())
        return dx, None


def activation(x, act):
    """act(x) elementwise (L.ACT_*)."""
    if act == L.ACT_NONE:
        return x
    return _ActFn.apply(x, act)


class _ResizeConcatFn(torch.autograd.Function):
    """cat([resize(p) for p in pieces], channels) with each bilinear resize (or plain copy when
    the size already matches) written straight into its channel slice (decoder_v8.py:152-156)."""

    @staticmethod
    def forward(ctx, size, align, *pieces):
        _require_cuda(*pieces)
        pieces = [_c(p) for p in pieces]
        n = pieces[0].shape[0]
        oh, ow = size
        widths = [p.shape[-1] for p in pieces]
        ct = sum(widths)
        out = torch.empty(n, oh, ow, ct, device=pieces[0].device, dtype=torch.float32)
        off = 0
        for p, wd in zip(pieces, widths):
            _, h, w, _ = p.shape
            if (h, w) == (oh, ow):
                _copy2d(p.view(-1, wd), out.view(-1, ct)[:, off:off + wd])
            else:
                L.call("mdemi_bilinear_fwd", p.data_ptr(), out.data_ptr() + 4 * off, n, h, w, wd, oh, ow, int(align),
                       0.0, 0.0, wd, ct, L.stream())
            off += wd
        ctx.shapes = [tuple(p.shape) for p in pieces]
        ctx.cfg = (oh, ow, align, ct)
        return out

    @staticmethod
    def backward(ctx, dy):
        oh, ow, align, ct = ctx.cfg
        dy = _c(dy)
        grads, off = [], 0
        for (n, h, w, wd) in ctx.shapes:
            g = torch.empty(n, h, w, wd, device=dy.device, dtype=torch.float32)
            if (h, w) == (oh, ow):
                _copy2d(dy.view(-1, ct)[:, off:off + wd], g.view(-1, wd))
            else:
                L.call("mdemi_bilinear_bwd", dy.data_ptr() + 4 * off, g.data_ptr(), n, h, w, wd, oh, ow, int(align),
                       0.0, 0.0, ct, wd, 0, L.stream())
            grads.append(g)
            off += wd
        return (None, None) + tuple(grads)


def resize_concat(pieces, size, align_corners=True):
    return _ResizeConcatFn.apply(tuple(size), align_corners, *pieces)


# ==========================================================================
# ODA2 ordered-swin2 ops (include/mdemi_ext.h, csrc/oda2.hip)
# ==========================================================================


class _PadReplicateFn(torch.autograd.Function):
    """Clamp-gather of an NHWC map to (OH, OW) with top/left offsets (pt, pl): replicate
    padding on any side and/or cropping.  Backward folds the gradient onto the source."""

    @staticmethod
    def forward(ctx, x, oh, ow, pt, pl):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n, oh, ow, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_pad_replicate", x.data_ptr(), y.data_ptr(), n, h, w, c, oh, ow, pt, pl, 0, L.stream())
        ctx.cfg = (n, h, w, c, oh, ow, pt, pl)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, oh, ow, pt, pl = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_pad_replicate", dy.data_ptr(), dx.data_ptr(), n, h, w, c, oh, ow, pt, pl, 1, L.stream())
        return dx, None, None, None, None


def pad_replicate_nhwc(x, top=0, bottom=0, left=0, right=0):
    """F.pad(..., mode='replicate') of an NHWC map's H / W (negative bottom/right crop)."""
    n, h, w, c = x.shape
    if top == bottom == left == right == 0:
        return x
    return _PadReplicateFn.apply(x, h + top + bottom, w + left + right, top, left)


def replicate_rows_nchw_no_grad(img, oh, ow):
    """Clamp-gather of an NCHW image (no gradient) as the NHWC map [N*C, H, W, 1]."""
    _require_cuda(img)
    img = _c(img)
    n, c, h, w = img.shape
    y = torch.empty(n, c, oh, ow, device=img.device, dtype=torch.float32)
    L.call("mdemi_pad_replicate", img.data_ptr(), y.data_ptr(), n * c, h, w, 1, oh, ow, 0, 0, 0, L.stream())
    return y


def resize_nchw_no_grad(img, oh, ow, align_corners=True):
    """Bilinear resize of an NCHW image that needs no gradient (the network input): the NHWC
    sweep over the [N*C, H, W, 1] view."""
    _require_cuda(img)
    img = _c(img)
    n, c, h, w = img.shape
    y = torch.empty(n, c, oh, ow, device=img.device, dtype=torch.float32)
    L.call("mdemi_bilinear_fwd", img.data_ptr(), y.data_ptr(), n * c, h, w, 1, oh, ow, int(align_corners), 0.0, 0.0,
           1, 1, L.stream())
    return y


class _WindowShuffleFn(torch.autograd.Function):
    """roll(-shift) + window_partition of an NHWC map into window-major rows [N*H*W, C]
    (oda2_red_order_swin2_decoder.py:83-85,103); backward is the scatter back."""

    @staticmethod
    def forward(ctx, x, ws, shift):
        _require_cuda(x)
        x = _c(x)
        n, h, w, c = x.shape
        y = torch.empty(n * h * w, c, device=x.device, dtype=torch.float32)
        L.call("mdemi_window_shuffle", x.data_ptr(), y.data_ptr(), None, n, h, w, c, ws, shift, 0, L.stream())
        ctx.cfg = (n, h, w, c, ws, shift)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, ws, shift = ctx.cfg
        dy = _c(dy)
        dx = torch.empty(n, h, w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_window_shuffle", dy.data_ptr(), dx.data_ptr(), None, n, h, w, c, ws, shift, 1, L.stream())
        return dx, None, None


class _WindowUnshuffleAddFn(torch.autograd.Function):
    """window_reverse + roll(+shift) of window-major rows back to NHWC, plus a residual in
    the natural layout (:126-131 `out + identity`)."""

    @staticmethod
    def forward(ctx, y_win, identity, ws, shift):
        _require_cuda(y_win, identity)
        y_win, identity = _c(y_win), _c(identity)
        n, h, w, c = identity.shape
        out = torch.empty_like(identity)
        L.call("mdemi_window_shuffle", y_win.data_ptr(), out.data_ptr(), identity.data_ptr(), n, h, w, c, ws, shift,
               1, L.stream())
        ctx.cfg = (n, h, w, c, ws, shift)
        return out

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, ws, shift = ctx.cfg
        dy = _c(dy)
        dwin = torch.empty(n * h * w, c, device=dy.device, dtype=torch.float32)
        L.call("mdemi_window_shuffle", dy.data_ptr(), dwin.data_ptr(), None, n, h, w, c, ws, shift, 0, L.stream())
        return dwin, dy, None, None


def window_shuffle(x_nhwc, ws, shift):
    return _WindowShuffleFn.apply(x_nhwc, ws, shift)


def window_unshuffle_add(y_win, identity_nhwc, ws, shift):
    return _WindowUnshuffleAddFn.apply(y_win, identity_nhwc, ws, shift)


def window_indices(idx_nhw, ws, shift):
    """int32 depth-index map [N, H, W] -> window-major [N*H*W] (rolled by -shift)."""
    idx = idx_nhw.to(torch.int32).contiguous()
    n, h, w = idx.shape
    out = torch.empty(n * h * w, device=idx.device, dtype=torch.int32)
    L.call("mdemi_window_shuffle_i32", idx.data_ptr(), out.data_ptr(), n, h, w, ws, shift, L.stream())
    return out


class _OrderedWindowAttnFn(torch.autograd.Function):
    """Per window and head: P = softmax(scale * drop(Q K^T) + E[idx_i - idx_j + n-1, h]),
    O = P V (oda2_red_order_swin2_decoder.py:111-122; attention dropout acts on the scaled
    scores before the bias, :117).  q/k/v are column slices [0,d) / [d,2d) / [2d,3d) of one
    window-major [nwin*T, 3d] buffer; QK^T, PV and their gradients are batched MFMA GEMMs
    (batch = (window, head)); the biased softmax and its backward (with the embedding
    gradient) are one sweep each.  Returns (O [nwin*T, d], P [nwin, heads, T, T])."""

    @staticmethod
    def forward(ctx, qkv, idx_win, table, cfg):
        nwin, T, heads, hd, num_emb, scale, p, seed = cfg
        _require_cuda(qkv, table)
        qkv = _c(qkv)
        d = heads * hd
        ld = 3 * d
        dev = qkv.device
        hs = T * T
        S = torch.empty(nwin, heads, T, T, device=dev, dtype=torch.float32)
        gemm(qkv, qkv, S, T, T, hd, lda=ld, ldb=ld, ldc=T, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
             batch=nwin * heads, a_bstride=T * ld, b_bstride=T * ld, c_bstride=heads * hs, a_off=0, b_off=d,
             inner=(heads, hd, hd, hs))
        if p > 0.0:
            _drop(S.data_ptr(), S.data_ptr(), S.numel(), p, seed)
        L.call("mdemi_ordered_softmax_fwd", S.data_ptr(), S.data_ptr(), L.ptr(idx_win), L.ptr(table), nwin, heads, T,
               num_emb, float(scale), L.stream())
        P = S
        out = torch.empty(nwin * T, d, device=dev, dtype=torch.float32)
        gemm(P, qkv, out, T, hd, T, lda=T, ldb=ld, ldc=d, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG,
             batch=nwin * heads, a_bstride=heads * hs, b_bstride=T * ld, c_bstride=T * d, b_off=2 * d,
             inner=(heads, hs, hd, hd))
        ctx.save_for_backward(qkv, P, idx_win)
        ctx.cfg = cfg
        ctx.has_table = table is not None
        ctx.set_materialize_grads(False)
        return out, P

    @staticmethod
    def backward(ctx, dout, dP_ext):
        qkv, P, idx_win = ctx.saved_tensors
        nwin, T, heads, hd, num_emb, scale, p, seed = ctx.cfg
        d = heads * hd
        ld = 3 * d
        hs = T * T
        dev = qkv.device
        dqkv = torch.empty_like(qkv)
        dP = torch.empty_like(P)
        if dout is not None:
            dout = _c(dout)
            gemm(dout, qkv, dP, T, T, hd, lda=d, ldb=ld, ldc=T, a_layout=L.L_KCONTIG, b_layout=L.L_KCONTIG,
                 batch=nwin * heads, a_bstride=T * d, b_bstride=T * ld, c_bstride=heads * hs, b_off=2 * d,
                 inner=(heads, hd, hd, hs))
            gemm(P, dout, dqkv, T, hd, T, lda=T, ldb=d, ldc=ld, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
                 batch=nwin * heads, a_bstride=heads * hs, b_bstride=T * d, c_bstride=T * ld, c_off=2 * d,
                 inner=(heads, hs, hd, hd))
            if dP_ext is not None:
                dP_ext = _c(dP_ext)
                L.call("mdemi_elementwise", L.EW_ADD, dP.data_ptr(), dP_ext.data_ptr(), dP.data_ptr(), dP.numel(),
                       0.0, 0.0, L.stream())
        else:
            dqkv[:, 2 * d:].zero_()
            if dP_ext is not None:
                _copy2d(_c(dP_ext).view(-1, T), dP.view(-1, T))
            else:
                dP.zero_()
        dtab = None
        lib = L.load()
        if ctx.has_table and ctx.needs_input_grad[2]:
            dtab = torch.empty(2 * num_emb - 1, heads, device=dev, dtype=torch.float32)
            ws = L.workspace(lib.mdemi_ordered_softmax_bwd_workspace_size(nwin, heads, num_emb), dev)
            wsp = ws.data_ptr()
        else:
            wsp = None
        L.check(lib.mdemi_ordered_softmax_bwd(P.data_ptr(), dP.data_ptr(), dP.data_ptr(), L.ptr(idx_win), L.ptr(dtab),
                                              nwin, heads, T, num_emb, float(scale), wsp, L.stream()),
                "ordered_softmax_bwd")
        dS = dP
        if p > 0.0:
            _drop(dS.data_ptr(), dS.data_ptr(), dS.numel(), p, seed)
        # dQ = dS K ; dK = dS^T Q
        gemm(dS, qkv, dqkv, T, hd, T, lda=T, ldb=ld, ldc=ld, a_layout=L.L_KCONTIG, b_layout=L.L_MNCONTIG,
             batch=nwin * heads, a_bstride=heads * hs, b_bstride=T * ld, c_bstride=T * ld, b_off=d, c_off=0,
             inner=(heads, hs, hd, hd))
        gemm(dS, qkv, dqkv, T, hd, T, lda=T, ldb=ld, ldc=ld, a_layout=L.L_MNCONTIG, b_layout=L.L_MNCONTIG,
             batch=nwin * heads, a_bstride=heads * hs, b_bstride=T * ld, c_bstride=T * ld, b_off=0, c_off=d,
             inner=(heads, hs, hd, hd))
        return dqkv, None, dtab, None


def ordered_window_attention(qkv_win, idx_win, table, nwin, T, heads, hd, num_emb, scale, p=0.0, training=False):
    p = float(p) if training else 0.0
    seed = _draw_seed(qkv_win.device) if p > 0.0 else None
    cfg = (nwin, T, heads, hd, int(num_emb), float(scale), p, seed)
    return _OrderedWindowAttnFn.apply(qkv_win, idx_win, table, cfg)


class _GluFn(torch.autograd.Function):
    """nn.GLU(dim=-1): x[..., :F] * sigmoid(x[..., F:])."""

    @staticmethod
    def forward(ctx, x):
        _require_cuda(x)
        x = _c(x)
        F2 = x.shape[-1]
        M = x.numel() // F2
        y = torch.empty(*x.shape[:-1], F2 // 2, device=x.device, dtype=torch.float32)
        L.call("mdemi_glu_fwd", x.data_ptr(), y.data_ptr(), M, F2 // 2, L.stream())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = _c(dy)
        F2 = x.shape[-1]
        dx = torch.empty_like(x)
        L.call("mdemi_glu_bwd", x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel() // F2, F2 // 2, L.stream())
        return dx


def glu(x):
    return _GluFn.apply(x)
