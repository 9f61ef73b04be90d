"""Tensor-level wrappers over the C ABI (libsdk_amd.so).

Activations are NHWC fp16 CUDA tensors ``[B, H, W, C]`` (tokens ``[B, N, C]`` are
the ``W = 1`` case).  A conv source may be a 2-tuple ``(a, b)`` meaning the
channel concat ``cat([a, b], -1)``, read zero-copy by the kernels.

There is no CPU or eager-PyTorch fallback: a non-CUDA tensor raises TypeError,
a library failure raises RuntimeError.
"""
from __future__ import annotations

import ctypes as C
import math

import torch

from . import _lib
from ._lib import (ACT_NONE, ACT_QUICK_GELU, AttentionArgs, XAttnArgs, XAttnLnArgs, FfArgs, TokenLinearArgs, ConvArgs, ConvPlanInfo, DdimArgs, GroupNormArgs,
                   OUT_GEGLU_F16, OUT_NCHW_F32, OUT_NHWC_F16, OUT_ROWS_F32, check, lib)

BK = 64          # K tile of the conv kernel (packed weight column padding)
BN = 128         # packed weight row padding (the kernels clamp reads beyond it)


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _need_cuda(t: torch.Tensor, what: str, dtype=torch.float16):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"sd_amd.{what}: expected a CUDA tensor (HIP path only, no CPU fallback)")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"sd_amd.{what}: expected {dtype}, got {t.dtype}")


# --------------------------------------------------------------------------- workspace

class _Workspace:
    """Growable scratch buffers (split-K slabs, GroupNorm partials), one per (device, lane).
    Calls of one lane are stream-ordered on one stream, so its buffer is safe to reuse;
    work issued concurrently on another stream must run under another lane
    (``with WORKSPACE.use_lane(i)``).

    A grown buffer is RETIRED, not freed: a HIP graph captured earlier holds the old
    pointer and writes through it on every replay, so its memory must stay owned by this
    workspace for the process lifetime (the superseded sizes sum to less than the final one
    when growth doubles; ``release_retired()`` is for callers that dropped every graph)."""

    def __init__(self):
        self.buf = {}
        self.retired = []
        self.lane = 0

    def release_retired(self):
        self.retired.clear()

    def use_lane(self, lane: int):
        import contextlib

        @contextlib.contextmanager
        def cm():
            prev, self.lane = self.lane, lane
            try:
                yield
            finally:
                self.lane = prev
        return cm()

    def counters(self, device) -> torch.Tensor:
        """The lane's per-tile arrival counters of in-launch split-K convs: zeroed once, and every launch
        leaves them zero (its last arrival resets each), so one fixed buffer serves every call of the lane."""
        key = (torch.device(device).index, self.lane, "cnt")
        c = self.buf.get(key)
        if c is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("sd_amd: tile counters must exist before graph capture (run one warm-up step)")
            c = torch.zeros(TILE_COUNTERS, dtype=torch.int32, device=device)
            self.buf[key] = c
        return c

    def get(self, nbytes: int, device) -> torch.Tensor:
        key = (torch.device(device).index, self.lane)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("sd_amd: workspace must be sized before graph capture (run one warm-up step)")
            if b is not None:
                self.retired.append(b)
                nbytes = max(nbytes, 2 * b.numel())       # geometric growth bounds the retired total
            b = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b


WORKSPACE = _Workspace()
TILE_COUNTERS = 16384     # sdk_amd.h SDK_TILE_COUNTERS


# --------------------------------------------------------------------------- sources

def _as_pair(x):
    if isinstance(x, tuple):
        a, b = x
        return a, b
    return x, None


def src_shape(x):
    a, b = _as_pair(x)
    B, H, W, C0 = a.shape
    return B, H, W, C0 + (b.shape[-1] if b is not None else 0)


def _fill_src(s: "_lib.ConvSrc", x, ksize, stride, pad, upsample, gn, silu):
    a, b = _as_pair(x)
    _need_cuda(a, "conv2d")
    B, H, W, C0 = a.shape
    if a.stride(3) != 1 or (H > 1 and a.stride(1) != W * a.stride(2)) or (B > 1 and a.stride(0) != H * a.stride(1)):
        raise ValueError("sd_amd.conv2d: source must be NHWC with contiguous channels and a uniform pixel stride")
    s.src0 = a.data_ptr()
    s.ld0 = a.stride(2) if a.dim() == 4 else a.stride(1)
    if b is not None:
        _need_cuda(b, "conv2d")
        s.src1 = b.data_ptr()
        s.ld1 = b.stride(2)
        s.c_split = C0
        s.cin = C0 + b.shape[-1]
    else:
        s.src1 = None
        s.ld1 = 0
        s.c_split = C0
        s.cin = C0
    s.h, s.w = H, W
    s.ksize, s.stride, s.pad, s.upsample = ksize, stride, pad, 1 if upsample else 0
    if gn is not None:
        s.gn_scale, s.gn_shift = gn[0].data_ptr(), gn[1].data_ptr()
    else:
        s.gn_scale = s.gn_shift = None
    s.silu = 1 if silu else 0
    return B, H, W


# --------------------------------------------------------------------------- packed weights

class PackedConv:
    """A conv / linear weight packed for the implicit-GEMM kernel.

    ``segments``: list of (weight [N, Cin, k, k] or [N, Cin], cin_src) — cin_src is
    the channel count of the NHWC source feeding that segment (>= Cin; extra
    channels get zero weights).  Packed layout: fp16 [roundup(N,128)][sum_s k*k*roundup(cin_src,64)],
    per segment 64-channel block major, then tap, then channel.  ``geglu`` interleaves the (x, gate) halves of a
    GEGLU projection in 32-row groups so one wave holds both.
    """

    def __init__(self, segments, bias=None, geglu=False, device="cuda"):
        cols, self.seg_geom = [], []
        n_out = None
        for w, cin_src in segments:
            w = w.detach().float()
            if w.dim() == 2:
                w = w[:, :, None, None]
            if w.dim() == 3:                      # Conv1d [N, Cin, 1]
                w = w[:, :, :, None]
            N, Cin, kh, kw = w.shape
            assert kh == kw, "square kernels only"
            if n_out is None:
                n_out = N
            assert N == n_out
            cin_pad = (cin_src + BK - 1) // BK * BK
            wp = torch.zeros(N, kh, kw, cin_pad, dtype=torch.float32, device=w.device)
            wp[:, :, :, :Cin] = w.permute(0, 2, 3, 1)
            # K order: 64-channel block major, tap minor (the kernels' K-step order)
            wp = wp.reshape(N, kh * kw, cin_pad // BK, BK).permute(0, 2, 1, 3)
            cols.append(wp.reshape(N, -1))
            self.seg_geom.append((kh, cin_src))
        Wt = torch.cat(cols, dim=1)
        b = bias.detach().float().clone() if bias is not None else None
        if geglu:
            inner = n_out // 2
            assert inner % 32 == 0
            idx = []
            for q in range(inner // 32):
                idx += list(range(32 * q, 32 * q + 32)) + list(range(inner + 32 * q, inner + 32 * q + 32))
            idx = torch.tensor(idx, device=Wt.device)
            Wt = Wt[idx]
            if b is not None:
                b = b[idx.to(b.device)]
        self.N = n_out
        self.geglu = geglu
        npad = (n_out + BN - 1) // BN * BN
        Wfull = torch.zeros(npad, Wt.shape[1], dtype=torch.float32, device=Wt.device)
        Wfull[:n_out] = Wt
        self.weight = Wfull.to(device=device, dtype=torch.float16).contiguous()
        self.k_total = self.weight.shape[1]
        self.bias = b.to(device=device, dtype=torch.float32).contiguous() if b is not None else None


class PerImageWeights:
    """Per-image GEMM weights for ``linear(..., n_img=)``: ``weight`` fp16 [batch, n_pad, k] (row n of
    image b's matrix, K contiguous; n_pad = roundup(n, 128)), so output rows of image b use matrix b
    (``sdk_conv_args.weight_batch_stride``).  The reassociated cross-attention's per-prompt K_h Wq_h and
    Wo_h V_h^T (openai_model/attention.py)."""

    def __init__(self, weight, n, bias=None):
        assert weight.dim() == 3 and weight.dtype == torch.float16 and weight.is_contiguous()
        assert weight.shape[1] % BN == 0 and weight.shape[2] % BK == 0 and n <= weight.shape[1]
        self.weight = weight
        self.N = n
        self.k_total = weight.shape[2]
        self.bias = bias
        self.geglu = False
        self.seg_geom = [(1, weight.shape[2])]
        self.w_batch_stride = weight.shape[1] * weight.shape[2]


def _conv_source_hash():
    import hashlib
    import os
    # SD_AMD_CONV_SOURCE: the conv.hip an A/B library (SD_AMD_LIB) was built from (tools only)
    src = os.environ.get("SD_AMD_CONV_SOURCE") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc",
                                                                "conv.hip")
    with open(src, "rb") as f:
        return hashlib.sha1(f.read()).hexdigest()[:16]


class _Autotune:
    """Per-shape choice of conv tile configuration and split-K, measured on the device.

    Enabled by ``enable()`` (UNetModel/AutoEncoderKL.prepare(autotune=True)); the
    first call of each distinct problem times every candidate (HIP events, 3 reps
    after a warm-up; SD_AMD_TUNE_REPS) and caches the fastest.  Never runs under graph capture."""
    VARIANTS = (2, 7, 6, 4, 3, 8, 9, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 31, 32, 33, 34, 35, 38, 40)
    # split -2: two K halves combined inside the launch (sdk_conv_args.split_inlaunch; LDS-DMA tile kernels)
    # (3 and 6: 80 256x256 tiles of a 16x16-level conv x 3 = 240 workgroups, one wave of the 256 CUs)
    SPLITS = (0, 1, 2, 3, 4, 6, 8, 12, 16, -2)
    # unsplit plans: M-panels per tile group (sdk_conv_args.tile_group_m; 1 = M-panel major)
    GROUPS = (1, 8, 16)

    def __init__(self):
        import os
        self.enabled = False
        self.table = {}
        self.timed = 0
        ev = os.environ.get("SD_AMD_TUNE_VARIANTS")       # candidate subset (benchmarking the tuner itself)
        if ev:
            self.VARIANTS = tuple(int(v) for v in ev.split(","))
        self.reps = int(os.environ.get("SD_AMD_TUNE_REPS", "3"))   # timed launches per candidate

    def enable(self, on=True):
        self.enabled = on

    def save(self, path):
        """Write the table as JSON (key tuple -> [variant_hint, split_k, tile_group_m]); a tuning cache
        like MIOpen's find-db: later runs load it and time nothing."""
        import json
        with open(path, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else None,
                       "conv_source": _conv_source_hash(),
                       "entries": [[list(k), list(v)] for k, v in sorted(self.table.items(), key=str)]}, f, indent=0)

    def load(self, path):
        import json
        with open(path) as f:
            d = json.load(f)
        if d.get("conv_source") != _conv_source_hash():
            return 0                     # tuned against other kernel code: re-time everything
        n = 0
        for k, v in d["entries"]:
            self.table[tuple(k)] = tuple(v)
            n += 1
        return n

    def key(self, a, pc, gn=False):
        s0, s1 = a.seg[0], a.seg[1]
        return (a.batch, a.ho, a.wo, a.cout, a.nseg, pc.k_total, a.out_mode, s0.cin, s0.h, s0.w, s0.ksize,
                s0.stride, s0.upsample, s0.c_split, int(bool(s0.gn_scale) or bool(s0.silu)),
                s1.cin if a.nseg > 1 else 0, int(gn), int(bool(a.weight_batch_stride)))

    def choose(self, a, pc, dev, gn=False):
        """``gn``: the output feeds a GroupNorm — candidates are timed emitting the statistics, and
        plans that cannot emit them are dropped (their GroupNorm would pay a statistics pass)."""
        key = self.key(a, pc, gn)
        hit = self.table.get(key)
        if hit is not None or not self.enabled or torch.cuda.is_current_stream_capturing():
            return hit
        cands = self.VARIANTS
        if a.nseg > 1 and (a.seg[1].gn_scale or a.seg[1].silu):
            self.table[key] = (0, 0)
            return self.table[key]
        if a.seg[0].gn_scale or a.seg[0].silu:
            # a transform prologue: the register-staged kernel or the skinny M <= 64 GEMM (SiLU on its A
            # fragments)
            cands = (0, 35)
        best, best_t = (0, 0), float("inf")
        info = ConvPlanInfo()
        stream = _stream()
        emit_any = False
        if gn:                           # is there a candidate at all that emits the statistics?
            for v in cands:
                for sp in self.SPLITS:
                    a.variant_hint = v + 1
                    set_split(a, sp, dev)
                    if lib().sdk_conv2d_plan(C.byref(a), C.byref(info)) == 0 and info.gn_chunks > 0:
                        emit_any = True
        for v in cands:
            for sp in self.SPLITS:
                a.variant_hint = v + 1
                set_split(a, sp, dev)
                if lib().sdk_conv2d_plan(C.byref(a), C.byref(info)) != 0:
                    continue
                if info.variant != v:
                    continue             # the forced variant does not apply: the planner's pick is timed once, as its own id
                if sp == 0 and info.split_k in self.SPLITS[1:]:
                    continue             # the automatic split equals an explicit candidate
                part = None
                if emit_any:
                    if info.gn_chunks == 0:
                        continue
                    part = torch.empty(a.batch, info.gn_chunks, a.cout, 2, dtype=torch.float32, device=dev)
                    a.gn_partial = part.data_ptr()
                else:
                    a.gn_partial = None
                if info.workspace_bytes > 0:
                    ws = WORKSPACE.get(info.workspace_bytes, dev)
                    a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel()
                for gm in (self.GROUPS if info.split_k == 1 else (0,)):
                    a.tile_group_m = gm
                    check(lib().sdk_conv2d(C.byref(a), stream), "conv2d(autotune)")
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(self.reps):
                        lib().sdk_conv2d(C.byref(a), stream)
                    e1.record()
                    e1.synchronize()
                    t = e0.elapsed_time(e1)
                    if t < best_t:
                        best_t, best = t, (v + 1, -2 if sp == -2 else info.split_k, gm)
        a.variant_hint, a.gn_partial, a.tile_group_m = 0, None, 0
        set_split(a, 0, dev)
        self.table[key] = best
        self.timed += 1
        if self.timed % 10 == 0:             # progress (a full re-tune takes minutes)
            import sys
            print(f"sd_amd autotune: {self.timed} conv problems timed", file=sys.stderr, flush=True)
        return best


AUTOTUNE = _Autotune()


def set_split(a, sp, dev):
    """split_k of a ConvArgs; ``sp == -2`` requests the in-launch combine of two K halves (its arrival
    counters: ``WORKSPACE.counters``)."""
    if sp == -2:
        a.split_k, a.split_inlaunch = 2, 1
        a.tile_counters = WORKSPACE.counters(dev).data_ptr()
    else:
        a.split_k, a.split_inlaunch, a.tile_counters = sp, 0, None


# tests / benchmarks: force one tile configuration on every conv call (None = planner / autotuner)
FORCE_VARIANT = None
# tests / benchmarks: M-panels per tile group of unsplit plans (sdk_conv_args.tile_group_m; None = library default)
TILE_GROUP_M = None


# GroupNorm statistics emitted by the producing conv (tensor attribute; see conv2d(gn_stats=True))
GN_ATTR = "_sd_gn_partial"
EMIT_GN_STATS = True      # tests / A/B: False = every GroupNorm runs its own statistics pass


def _claim(out):
    """A caller-supplied ``out`` is about to be overwritten through the C ABI, which does not move
    torch's version counter: drop any GroupNorm statistics a previous producer attached to it, so
    only the plan that writes it now can attach (fresh) ones."""
    if out is not None and hasattr(out, GN_ATTR):
        delattr(out, GN_ATTR)
    return out


# The LDS-DMA conv kernels address a source through a buffer resource (31-bit byte offsets); a source
# of >= 2 GiB (the VAE decoder's 256-channel 512x512 maps at B=16: 2.15 GB) would push the plan onto
# the register-staged kernel (~500 vs ~800 TFLOP/s).  Such convs run as batch chunks under the limit
# (SD_AMD_CONV_CHUNK_LIMIT overrides it: A/B only).
BUF_LIMIT = int(__import__("os").environ.get("SD_AMD_CONV_CHUNK_LIMIT", "2147483647"))


def _src_bytes(x):
    a, b = _as_pair(x)
    B, H, W, _ = a.shape
    ld = max(a.stride(2), b.stride(2) if b is not None else 0)
    return B * H * W * ld * 2


def _bslice(t, b0, b1):
    if t is None:
        return None
    if isinstance(t, tuple):
        return tuple(_bslice(u, b0, b1) for u in t)
    return t[b0:b1]


def _conv2d_batch_chunks(pc, x, seg2, gn, row_bias, residual, out, B, kw):
    big = max(_src_bytes(x), _src_bytes(seg2[0]) if seg2 is not None else 0)
    n = -(-big // BUF_LIMIT)
    while big * 1.0 / n >= BUF_LIMIT or B % n:
        n += 1
        if n >= B:
            n = B
            break
    cb = B // n
    outs = []
    for b0 in range(0, B, cb):
        b1 = min(B, b0 + cb)
        s2 = None if seg2 is None else (_bslice(seg2[0], b0, b1), _bslice(seg2[1], b0, b1), seg2[2])
        rb = None if row_bias is None else (row_bias[0][b0:b1], row_bias[1])
        outs.append(conv2d(pc, _bslice(x, b0, b1), seg2=s2, gn=_bslice(gn, b0, b1), row_bias=rb,
                           residual=_bslice(residual, b0, b1), out=None if out is None else out[b0:b1], **kw))
    full = out if out is not None else torch.cat(outs, 0)
    parts = [getattr(o, GN_ATTR, None) for o in outs]
    if all(pp is not None for pp in parts) and len({pp[1] for pp in parts}) == 1:
        setattr(full, GN_ATTR, (torch.cat([pp[0] for pp in parts], 0), parts[0][1], full._version))
    return full


def conv2d(pc: PackedConv, x, *, ksize=None, stride=1, pad=None, pad_end=0, upsample=False, gn=None, silu=False,
           seg2=None, bias=True, row_bias=None, residual=None, out_mode=OUT_NHWC_F16, out=None,
           variant=None, split_k=None, act=ACT_NONE, gn_stats=False):
    """Run the implicit-GEMM conv.  ``seg2`` = (x2, gn2, silu2) adds a fused 1x1 K segment.
    ``pad_end`` adds zero rows/cols after the source (asymmetric (0,1,0,1) padding).
    ``row_bias`` = (fp32 tensor [B, ld], column offset) — the per-(batch, channel) add.
    ``variant`` / ``split_k`` force a kernel configuration (benchmarks; default: planner
    or autotuner).  ``gn_stats``: the output feeds a GroupNorm — when the chosen plan can, the
    epilogue also emits its per-chunk channel statistics (attached to the returned tensor,
    consumed by ``group_norm``, which then skips its statistics pass)."""
    _claim(out)
    B0 = _as_pair(x)[0].shape[0]
    if B0 > 1 and (_src_bytes(x) >= BUF_LIMIT or (seg2 is not None and _src_bytes(seg2[0]) >= BUF_LIMIT)):
        if out is None:
            a0 = _as_pair(x)[0]
            lh, lw = (2 * a0.shape[1], 2 * a0.shape[2]) if upsample else (a0.shape[1], a0.shape[2])
            k_ = pc.seg_geom[0][0] if ksize is None else ksize
            p_ = k_ // 2 if pad is None else pad
            Ho = (lh + 2 * p_ + pad_end - k_) // stride + 1
            Wo = (lw + 2 * p_ + pad_end - k_) // stride + 1
            shape = {OUT_NHWC_F16: (B0, Ho, Wo, pc.N), OUT_GEGLU_F16: (B0, Ho, Wo, pc.N // 2),
                     OUT_NCHW_F32: (B0, pc.N, Ho, Wo)}.get(out_mode, (B0, Ho, Wo, pc.N))
            dt = torch.float16 if out_mode in (OUT_NHWC_F16, OUT_GEGLU_F16) else torch.float32
            out = torch.empty(shape, dtype=dt, device=a0.device)
        kw = dict(ksize=ksize, stride=stride, pad=pad, pad_end=pad_end, upsample=upsample, silu=silu, bias=bias,
                  out_mode=out_mode, variant=variant, split_k=split_k, act=act, gn_stats=gn_stats)
        return _conv2d_batch_chunks(pc, x, seg2, gn, row_bias, residual, out, B0, kw)
    a = ConvArgs()
    k0 = pc.seg_geom[0][0] if ksize is None else ksize
    if pad is None:
        pad = k0 // 2
    B, H, W = _fill_src(a.seg[0], x, k0, stride, pad, upsample, gn, silu)
    a.seg[0].pad_end = pad_end
    lh, lw = (2 * H, 2 * W) if upsample else (H, W)
    Ho = (lh + 2 * pad + pad_end - k0) // stride + 1
    Wo = (lw + 2 * pad + pad_end - k0) // stride + 1
    a.nseg = 1
    if seg2 is not None:
        x2, gn2, silu2 = seg2
        _fill_src(a.seg[1], x2, 1, 1, 0, False, gn2, silu2)
        a.nseg = 2
    a.batch, a.ho, a.wo, a.cout = B, Ho, Wo, pc.N
    a.act = act
    a.weight = pc.weight.data_ptr()
    a.k_total = pc.k_total
    a.weight_batch_stride = getattr(pc, "w_batch_stride", 0)
    a.bias = pc.bias.data_ptr() if (bias and pc.bias is not None) else None
    if row_bias is not None:
        rb, off = row_bias
        a.row_bias = rb.data_ptr() + 4 * off
        a.row_bias_ld = rb.stride(0)
    dev = (x[0] if isinstance(x, tuple) else x).device
    if out is None:
        if out_mode == OUT_NHWC_F16:
            out = torch.empty(B, Ho, Wo, pc.N, dtype=torch.float16, device=dev)
        elif out_mode == OUT_GEGLU_F16:
            out = torch.empty(B, Ho, Wo, pc.N // 2, dtype=torch.float16, device=dev)
        elif out_mode == OUT_NCHW_F32:
            out = torch.empty(B, pc.N, Ho, Wo, dtype=torch.float32, device=dev)
        else:
            out = torch.empty(B, Ho, Wo, pc.N, dtype=torch.float32, device=dev)
    a.out = out.data_ptr()
    a.out_ld = out.shape[-1] if out_mode != OUT_NCHW_F32 else 0
    a.out_mode = out_mode
    if residual is not None:
        _need_cuda(residual, "conv2d residual")
        a.residual = residual.data_ptr()
        a.res_ld = residual.shape[-1]
    want_gn = gn_stats and EMIT_GN_STATS and out_mode == OUT_NHWC_F16
    tuned = AUTOTUNE.choose(a, pc, dev, want_gn) if (AUTOTUNE.enabled or AUTOTUNE.table) else None
    if tuned is not None:
        a.variant_hint = tuned[0]
        set_split(a, tuned[1], dev)
        a.tile_group_m = tuned[2] if len(tuned) > 2 else 0
    if variant is None:
        variant = FORCE_VARIANT
    if variant is not None:
        if variant + 1 != a.variant_hint:
            # a forced configuration: the tuned split / tile order belong to the tuned variant (an in-launch
            # split may not even exist for this one) -> the planner's split for the forced variant
            set_split(a, 0, dev)
            a.tile_group_m = 0
        a.variant_hint = variant + 1
    if split_k is not None:
        set_split(a, split_k, dev)    # -2: the in-launch combine of two K halves
    if TILE_GROUP_M is not None:
        a.tile_group_m = TILE_GROUP_M
    info = ConvPlanInfo()
    check(lib().sdk_conv2d_plan(C.byref(a), C.byref(info)), "conv2d_plan")
    if info.workspace_bytes > 0:
        ws = WORKSPACE.get(info.workspace_bytes, dev)
        a.workspace = ws.data_ptr()
        a.workspace_bytes = ws.numel()
    part = None
    if want_gn and info.gn_chunks > 0 and out.shape[-1] == pc.N:
        part = torch.empty(B, info.gn_chunks, pc.N, 2, dtype=torch.float32, device=dev)
        a.gn_partial = part.data_ptr()
    if PROFILER.active:
        # algorithmic HBM bytes: each source tensor, the weights and the output once (+ residual)
        nb = sum(t.numel() * 2 for t in _as_pair(x) if t is not None) + pc.N * pc.k_total * 2
        if seg2 is not None:
            nb += sum(t.numel() * 2 for t in _as_pair(seg2[0]) if t is not None)
        nb += out.numel() * out.element_size() + (residual.numel() * 2 if residual is not None else 0)
        PROFILER.begin("conv", info, shape=(B * Ho * Wo, pc.N, pc.k_total, info.variant, info.split_k), nbytes=nb)
    check(lib().sdk_conv2d(C.byref(a), _stream()), "conv2d")
    if PROFILER.active:
        PROFILER.end()
    if part is not None:
        # the statistics describe `out` as written now: group_norm ignores them once the tensor has
        # been modified in place (its version counter moved)
        setattr(out, GN_ATTR, (part, info.gn_chunks, out._version))
    return out


def linear(pc: PackedConv, x2d, *, silu=False, residual=None, out_mode=OUT_NHWC_F16, out=None, bias=True,
           act=ACT_NONE, n_img=None):
    """Token GEMM: x2d [M, K] fp16 → [M, N]; a 1x1 conv over an M x 1 image.  ``silu`` applies to
    the input (prologue), ``act`` to the output (epilogue, before the residual).  ``n_img``: rows per
    image, for a ``PerImageWeights`` pc (the GEMM runs as M / n_img images of n_img x 1)."""
    _claim(out)
    M = x2d.shape[0]
    nb, rows = (1, M) if n_img is None else (M // n_img, n_img)
    assert nb * rows == M
    if isinstance(pc, PerImageWeights):
        assert n_img is not None and nb == pc.weight.shape[0], "per-image weights: n_img must split M by image"
    x4 = x2d.view(nb, rows, 1, x2d.shape[-1]) if x2d.stride(-1) == 1 and x2d.is_contiguous() else None
    if x4 is None:
        x4 = x2d.as_strided((nb, rows, 1, x2d.shape[1]), (rows * x2d.stride(0), x2d.stride(0), x2d.stride(0), 1))
    res4 = residual.view(nb, rows, 1, residual.shape[-1]) if residual is not None else None
    y = conv2d(pc, x4, ksize=1, pad=0, silu=silu, residual=res4, out_mode=out_mode, bias=bias,
               out=None if out is None else out.view(nb, rows, 1, out.shape[-1]), act=act)
    return y.view(M, y.shape[-1])


def segment_softmax(s, nseg, seglen, scale, ld_p=None, out=None):
    """p = softmax over each of the ``nseg`` ``seglen``-column segments of scale * s (fp32 [M, ld] →
    fp16 [M, ld_p], columns from nseg*seglen zero): the reassociated cross-attention's softmax."""
    _need_cuda(s, "segment_softmax", torch.float32)
    assert s.dtype == torch.float32 and s.stride(-1) == 1
    M = s.shape[0]
    ld_p = ld_p or (nseg * seglen + BK - 1) // BK * BK
    if out is None:
        out = torch.empty(M, ld_p, dtype=torch.float16, device=s.device)
    check(lib().sdk_segment_softmax(s.data_ptr(), s.stride(0), out.data_ptr(), out.stride(0), M, nseg, seglen,
                                    float(scale), _stream()), "segment_softmax")
    return out


# --------------------------------------------------------------------------- normalisation

def _gn_args(x):
    a0, a1 = _as_pair(x)
    _need_cuda(a0, "group_norm")
    B, H, W, Ch = src_shape(x)
    args = GroupNormArgs()
    args.src0 = a0.data_ptr()
    args.ld0 = a0.stride(2)
    if a1 is not None:
        args.src1 = a1.data_ptr()
        args.ld1 = a1.stride(2)
    args.c_split = a0.shape[-1]
    args.batch, args.hw, args.channels = B, H * W, Ch
    return args, (B, H, W, Ch), a0.device


# zero-bordered GN+SiLU outputs for pad-0 3x3 convs (mask-free gather); 0 = the masked pad-1 path
PREPAD = 1


def gn_conv_pad():
    """(pad written by group_norm_apply, pad of the 3x3 conv that consumes it)."""
    return (1, 0) if PREPAD else (0, 1)


def group_norm_apply(x, gn, silu=True, out=None, pad=0):
    """y = silu?(x*scale + shift) — the normalised (possibly concatenated) input, contiguous NHWC.
    ``pad`` > 0 writes it into a zero-bordered [B, H+2pad, W+2pad, C] image for a pad-0 3x3 conv."""
    args, (B, H, W, Ch), dev = _gn_args(x)
    args.scale, args.shift = gn[0].data_ptr(), gn[1].data_ptr()
    y = _claim(out) if out is not None else torch.empty(B, H + 2 * pad, W + 2 * pad, Ch, dtype=torch.float16,
                                                          device=dev)
    if PROFILER.active:
        PROFILER.begin("gn_apply", None)
    if pad:
        check(lib().sdk_group_norm_apply_padded(C.byref(args), 1 if silu else 0, _ptr(y), Ch, H, W, pad, _stream()),
              "group_norm_apply_padded")
    else:
        check(lib().sdk_group_norm_apply(C.byref(args), 1 if silu else 0, _ptr(y), Ch, _stream()),
              "group_norm_apply")
    if PROFILER.active:
        PROFILER.end()
    return y


def group_norm_apply_ex(x, gn, silu=True, post_bias=None, residual=None):
    """y = silu?(x*scale + shift) + post_bias[b, c] + residual (DDPM C1 post-activation GroupNorm)."""
    args, (B, H, W, Ch), dev = _gn_args(x)
    args.scale, args.shift = gn[0].data_ptr(), gn[1].data_ptr()
    y = torch.empty(B, H, W, Ch, dtype=torch.float16, device=dev)
    pb_ld = 0
    if post_bias is not None:
        _need_cuda(post_bias, "group_norm_apply_ex post_bias", torch.float32)
        pb_ld = post_bias.stride(0)
    res_ld = 0
    if residual is not None:
        _need_cuda(residual, "group_norm_apply_ex residual")
        res_ld = residual.shape[-1]
    if PROFILER.active:
        PROFILER.begin("gn_apply", None)
    check(lib().sdk_group_norm_apply_ex(C.byref(args), 1 if silu else 0, _ptr(post_bias), pb_ld, _ptr(residual),
                                        res_ld, _ptr(y), Ch, _stream()), "group_norm_apply_ex")
    if PROFILER.active:
        PROFILER.end()
    return y


def upsample_bilinear2x(x):
    """F.interpolate(scale_factor=2, mode='bilinear', align_corners=True) on NHWC fp16."""
    _need_cuda(x, "upsample_bilinear2x")
    x = x.contiguous()
    B, H, W, Cc = x.shape
    y = torch.empty(B, 2 * H, 2 * W, Cc, dtype=torch.float16, device=x.device)
    check(lib().sdk_upsample_bilinear2x(_ptr(x), _ptr(y), B, H, W, Cc, _stream()), "upsample_bilinear2x")
    return y


def upsample_nearest2x_padded(x, pad=1):
    """Nearest-x2 upsample of NHWC fp16 x into a zero-bordered [B, 2H + 2pad, 2W + 2pad, C] image (the UNet
    Upsample's interpolate; its 3x3 conv then runs with pad 0 on the unmasked linear issue)."""
    _need_cuda(x, "upsample_nearest2x_padded")
    B, H, W, Cc = x.shape
    if x.stride(-1) != 1 or x.stride(1) != W * x.stride(2) or x.stride(0) != H * x.stride(1):
        x = x.contiguous()
    y = torch.empty(B, 2 * H + 2 * pad, 2 * W + 2 * pad, Cc, dtype=torch.float16, device=x.device)
    check(lib().sdk_upsample_nearest2x_padded(_ptr(x), x.stride(2), _ptr(y), B, H, W, Cc, pad, _stream()),
          "upsample_nearest2x_padded")
    return y


def gelu(x):
    """Exact (erf) GELU, fp16."""
    _need_cuda(x, "gelu")
    x = x.contiguous()
    y = torch.empty_like(x)
    check(lib().sdk_gelu(_ptr(x), _ptr(y), x.numel(), _stream()), "gelu")
    return y


def group_norm_silu(x, gamma, beta, eps, groups=32):
    """GroupNorm + SiLU materialised once (stats pass + apply pass) — the input of a 3x3 conv."""
    return group_norm_apply(x, group_norm_affine(x, gamma, beta, eps, groups), silu=True)


def group_norm_scale_shift(x, gamma, beta, eps, groups=32):
    """Per-(batch, channel) fp32 (scale, shift) [B, C] of GroupNorm(x) from the statistics its producing
    convs emitted (else a statistics pass) — for a 3x3 conv that applies GroupNorm + SiLU to its own
    prologue (``conv2d(gn=(scale, shift), silu=True)`` on the register-staged kernel), so the normalised
    tensor is never written (``sdk_group_norm_finalize``)."""
    args, (B, H, W, Ch), dev = _gn_args(x)
    args.groups, args.eps = groups, eps
    args.gamma, args.beta = gamma.data_ptr(), beta.data_ptr()
    scale = torch.empty(B, Ch, dtype=torch.float32, device=dev)
    shift = torch.empty(B, Ch, dtype=torch.float32, device=dev)
    args.scale, args.shift = scale.data_ptr(), shift.data_ptr()
    ws = WORKSPACE.get(lib().sdk_group_norm_workspace(B, H * W, Ch), dev)
    args.workspace, args.workspace_bytes = ws.data_ptr(), ws.numel()
    srcs = [t for t in _as_pair(x) if t is not None]
    parts = [getattr(t, GN_ATTR, None) for t in srcs]
    parts = [pp if pp is not None and pp[2] == t._version else None for pp, t in zip(parts, srcs)]
    p0 = p1 = None
    n0 = n1 = 0
    if all(pp is not None for pp in parts):
        (p0, n0, _) = parts[0]
        if len(parts) > 1:
            (p1, n1, _) = parts[1]
    if PROFILER.active:
        PROFILER.begin("group_norm", None)
    check(lib().sdk_group_norm_finalize(C.byref(args), _ptr(p0), n0, _ptr(p1), n1, _stream()), "group_norm_finalize")
    if PROFILER.active:
        PROFILER.end()
    return scale, shift


def group_norm_affine(x, gamma, beta, eps, groups=32):
    """Per-(batch, channel) (scale, shift) fp32 [B, C] of GroupNorm(x) for the conv prologue."""
    a0, a1 = _as_pair(x)
    _need_cuda(a0, "group_norm")
    B, H, W, Ch = src_shape(x)
    args = GroupNormArgs()
    args.src0 = a0.data_ptr()
    args.ld0 = a0.stride(2)
    if a1 is not None:
        args.src1 = a1.data_ptr()
        args.ld1 = a1.stride(2)
    args.c_split = a0.shape[-1]
    args.batch, args.hw, args.channels, args.groups, args.eps = B, H * W, Ch, groups, eps
    args.gamma = gamma.data_ptr()
    args.beta = beta.data_ptr()
    scale = torch.empty(B, Ch, dtype=torch.float32, device=a0.device)
    shift = torch.empty(B, Ch, dtype=torch.float32, device=a0.device)
    args.scale, args.shift = scale.data_ptr(), shift.data_ptr()
    need = lib().sdk_group_norm_workspace(B, H * W, Ch)
    ws = WORKSPACE.get(need, a0.device)
    args.workspace, args.workspace_bytes = ws.data_ptr(), ws.numel()
    if PROFILER.active:
        PROFILER.begin("group_norm", None)
    check(lib().sdk_group_norm_affine(C.byref(args), _stream()), "group_norm_affine")
    if PROFILER.active:
        PROFILER.end()
    return scale, shift


def group_norm(x, gamma, beta, eps, groups=32, silu=True, pad=0, out=None):
    """GroupNorm (+ SiLU) end to end in one C call: statistics and apply, written contiguous or
    zero-bordered (``pad``) for a pad-0 3x3 conv.  At the UNet's small levels one fused launch;
    elsewhere the statistics pass then the apply pass (``sdk_group_norm``)."""
    args, (B, H, W, Ch), dev = _gn_args(x)
    args.groups, args.eps = groups, eps
    args.gamma, args.beta = gamma.data_ptr(), beta.data_ptr()
    scale = torch.empty(B, Ch, dtype=torch.float32, device=dev)
    shift = torch.empty(B, Ch, dtype=torch.float32, device=dev)
    args.scale, args.shift = scale.data_ptr(), shift.data_ptr()
    ws = WORKSPACE.get(lib().sdk_group_norm_workspace(B, H * W, Ch), dev)
    args.workspace, args.workspace_bytes = ws.data_ptr(), ws.numel()
    y = _claim(out) if out is not None else torch.empty(B, H + 2 * pad, W + 2 * pad, Ch, dtype=torch.float16,
                                                          device=dev)
    # statistics the producing convs emitted (every source must carry them)
    srcs = [t for t in _as_pair(x) if t is not None]
    parts = [getattr(t, GN_ATTR, None) for t in srcs]
    parts = [pp if pp is not None and pp[2] == t._version else None for pp, t in zip(parts, srcs)]
    p0 = p1 = None
    n0 = n1 = 0
    if all(pp is not None for pp in parts):
        (p0, n0, _) = parts[0]
        if len(parts) > 1:
            (p1, n1, _) = parts[1]
    if PROFILER.active:
        PROFILER.begin("group_norm", None)
    check(lib().sdk_group_norm(C.byref(args), 1 if silu else 0, _ptr(y), y.shape[-1], H, W, pad, _ptr(p0), n0,
                               _ptr(p1), n1, _stream()), "group_norm")
    if PROFILER.active:
        PROFILER.end()
    return y


def layer_norm(x2d, gamma, beta, eps=1e-5, out=None):
    _need_cuda(x2d, "layer_norm")
    M, Cc = x2d.shape
    y = _claim(out) if out is not None else torch.empty(M, Cc, dtype=torch.float16, device=x2d.device)
    if PROFILER.active:
        PROFILER.begin("layer_norm", None)
    check(lib().sdk_layer_norm(_ptr(x2d), _ptr(y), M, Cc, x2d.stride(0), y.stride(0), _ptr(gamma), _ptr(beta),
                               C.c_float(eps), _stream()), "layer_norm")
    if PROFILER.active:
        PROFILER.end()
    return y


# --------------------------------------------------------------------------- device calibration

def probe_peaks(reps=3):
    """Measured dense fp16 MFMA rate (both MFMA shapes, random operands, every CU busy) and HBM copy
    rate of this device (sdk_probe_*; HIP events, best of ``reps``) — the achievable ceilings next to
    the spec peaks the bench's roofline is quoted against."""
    dev = torch.device("cuda", torch.cuda.current_device())
    seed = torch.randn(32768, device=dev).half()
    nsm = torch.cuda.get_device_properties(dev).multi_processor_count
    sink = torch.empty(4 * nsm * 4, dtype=torch.float32, device=dev)
    out = {}
    # 2 or 4 workgroups of 4 waves per CU (2 / 4 waves per SIMD): the faster is the ceiling
    for m16, iters, name in ((1, 40000, "mfma_16x16x32_f16_tflops"), (0, 20000, "mfma_32x32x16_f16_tflops")):
        top = 0.0
        for blocks in (2 * nsm, 4 * nsm):
            check(lib().sdk_probe_mfma(m16, blocks, 200, _ptr(seed), _ptr(sink), _stream()), "probe_mfma")
            best = float("inf")
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                check(lib().sdk_probe_mfma(m16, blocks, iters, _ptr(seed), _ptr(sink), _stream()), "probe_mfma")
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1))
            top = max(top, lib().sdk_probe_mfma_flops(m16, blocks, iters) / (best * 1e-3) / 1e12)
        out[name] = round(top, 1)
    # HBM: a 1 GiB copy (read + write counted), the best of a few shapes — loads in flight per thread,
    # non-temporal or default policy, workgroups per CU (the fastest is the device's streaming ceiling)
    nbytes = 1 << 30
    src = torch.empty(nbytes // 2, dtype=torch.float16, device=dev).normal_()
    dst = torch.empty_like(src)
    best_gbs, best_mode = 0.0, 0
    for mode in (0, 1, 2, 3, 1 | (8 << 2), 3 | (8 << 2), 1 | (32 << 2), 3 | (32 << 2), 256, 257, 258, 259):
        check(lib().sdk_probe_copy_ex(_ptr(src), _ptr(dst), nbytes, mode, _stream()), "probe_copy")
        best = float("inf")
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            check(lib().sdk_probe_copy_ex(_ptr(src), _ptr(dst), nbytes, mode, _stream()), "probe_copy")
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        gbs = 2 * nbytes / (best * 1e-3) / 1e9
        if gbs > best_gbs:
            best_gbs, best_mode = gbs, mode
    out["hbm_copy_gbs"] = round(best_gbs, 1)
    out["hbm_copy_mode"] = {"loads_in_flight": 8 if best_mode & 1 else 4, "nontemporal": bool(best_mode & 2),
                            "form": "flat one pass" if best_mode & 256 else "grid-stride",
                            "workgroups_per_cu": None if best_mode & 256 else ((best_mode >> 2) & 63) or 16}
    del src, dst
    return out


# --------------------------------------------------------------------------- attention

def attention(q, k, v, *, batch, heads, nq, nk, head_dim, scale, out=None, causal=False):
    """q/k/v: 2-D fp16 views [batch*n, ld] (head h at columns h*head_dim...); ``causal`` masks
    key j > query i."""
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _need_cuda(t, "attention " + n)
    if out is None:
        out = torch.empty(batch * nq, heads * head_dim, dtype=torch.float16, device=q.device)
    _claim(out)
    a = AttentionArgs()
    a.q, a.k, a.v, a.o = q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr()
    a.q_ld, a.k_ld, a.v_ld, a.o_ld = q.stride(0), k.stride(0), v.stride(0), out.stride(0)
    a.batch, a.heads, a.nq, a.nk, a.head_dim, a.scale = batch, heads, nq, nk, head_dim, scale
    a.causal = 1 if causal else 0
    if PROFILER.active:
        PROFILER.begin("attention", (batch, heads, nq, nk, head_dim))
    check(lib().sdk_attention(C.byref(a), _stream()), "attention")
    if PROFILER.active:
        PROFILER.end()
    return out


def cross_attention_block_supported(channels, head_dim, nk, n_img):
    return bool(lib().sdk_cross_attention_block_supported(channels, head_dim, nk, n_img))


# the block's projection weights in the fragment-packed layout (sdk_xattn_pack_weight: whole 128-B lines per weight
# fetch); False = the row layout (A/B only, same bits)
XATTN_PACKED_W = True


def xattn_packed_weight(pc: PackedConv):
    """The fragment-packed copy of a channels x channels PackedConv for the cross-attention kernel, made once
    and kept on the PackedConv (not inside a graph capture: the first eager evaluation makes it)."""
    pk = getattr(pc, "_xattn_pk", None)
    if pk is None:
        Cc = pc.N
        pk = torch.empty(Cc * Cc, dtype=torch.float16, device=pc.weight.device)
        check(lib().sdk_xattn_pack_weight(pc.weight.data_ptr(), pc.k_total, pk.data_ptr(), Cc, _stream()),
              "xattn_pack_weight")
        pc._xattn_pk = pk
    return pk


def cross_attention_block(t, kv, pc_q: PackedConv, pc_o: PackedConv, *, batch, n_img, nk, heads, head_dim, scale,
                          residual=None, out=None, norm_in=None, norm_out=None, out_ln=None):
    """One-kernel cross-attention block on a cached context K|V: ``to_out(attn(to_q(t), K, V)) + residual``.
    t / residual: [batch*n_img, C] fp16; kv: [batch*nk, >= 2C] fp16 (K | V).

    ``norm_in`` = (gamma, beta, eps): ``t`` is the LayerNorm's INPUT and is normalised inside the
    kernel (BasicTransformerBlock.norm2); ``norm_out`` = (gamma, beta, eps): also returns
    LayerNorm(out) (norm3) — the result is then ``(out, out_ln)``.  Both match ``layer_norm``
    bit for bit."""
    Cc = heads * head_dim
    for x, n in ((t, "t"), (kv, "kv")):
        _need_cuda(x, "cross_attention_block " + n)
    if pc_q.k_total != Cc or pc_o.k_total != Cc or pc_q.N != Cc or pc_o.N != Cc:
        raise ValueError("sd_amd.cross_attention_block: to_q / to_out must be channels x channels")
    if out is None:
        out = torch.empty(batch * n_img, Cc, dtype=torch.float16, device=t.device)
    _claim(out)
    _claim(out_ln)
    a = XAttnArgs()
    a.t, a.kv, a.wq, a.wo = t.data_ptr(), kv.data_ptr(), pc_q.weight.data_ptr(), pc_o.weight.data_ptr()
    packed = XATTN_PACKED_W and (not torch.cuda.is_current_stream_capturing() or
                                 (hasattr(pc_q, "_xattn_pk") and hasattr(pc_o, "_xattn_pk")))
    if packed:
        a.wq, a.wo = xattn_packed_weight(pc_q).data_ptr(), xattn_packed_weight(pc_o).data_ptr()
    a.bias = pc_o.bias.data_ptr() if pc_o.bias is not None else None
    a.res = residual.data_ptr() if residual is not None else None
    a.out = out.data_ptr()
    a.t_ld, a.kv_ld, a.w_ld = t.stride(0), kv.stride(0), 0 if packed else Cc
    a.res_ld = residual.stride(0) if residual is not None else 0
    a.out_ld = out.stride(0)
    a.batch, a.n_img, a.nk, a.channels, a.head_dim, a.scale = batch, n_img, nk, Cc, head_dim, scale
    if PROFILER.active:
        # FLOPs of the three products it replaces (2 projections + attention core)
        PROFILER.begin("cross_attention_block", None)
        PROFILER._cur = PROFILER._cur[:2] + (4.0 * batch * n_img * Cc * Cc + 4.0 * batch * n_img * nk * Cc,) + \
            PROFILER._cur[3:]
    if norm_in is None and norm_out is None:
        check(lib().sdk_cross_attention_block(C.byref(a), _stream()), "cross_attention_block")
    else:
        ln = XAttnLnArgs()
        if norm_in is not None:
            ln.in_gamma, ln.in_beta, ln.in_eps = norm_in[0].data_ptr(), norm_in[1].data_ptr(), norm_in[2]
        if norm_out is not None:
            if out_ln is None:
                out_ln = torch.empty_like(out)
            ln.out_gamma, ln.out_beta, ln.out_eps = norm_out[0].data_ptr(), norm_out[1].data_ptr(), norm_out[2]
            ln.out_ln, ln.out_ln_ld = out_ln.data_ptr(), out_ln.stride(0)
        check(lib().sdk_cross_attention_block_ln(C.byref(a), C.byref(ln), _stream()), "cross_attention_block")
    if PROFILER.active:
        PROFILER.end()
    return (out, out_ln) if norm_out is not None else out


def ff_supported(channels, features):
    return bool(lib().sdk_ff_supported(channels, features))


class PackedFF:
    """The GEGLU FeedForward's weights packed once for ``feed_forward`` (sdk_ff_pack): proj (Linear(C, 2F):
    rows [0, F) = a, [F, 2F) = gate) and the output Linear(F, C)."""

    def __init__(self, w1, b1, w2, b2, device):
        F2, Cc = w1.shape
        self.channels, self.features = Cc, F2 // 2
        if not ff_supported(Cc, self.features):
            raise ValueError(f"sd_amd.PackedFF: unsupported shape channels={Cc} features={self.features}")
        w1h = w1.detach().to(device=device, dtype=torch.float16).contiguous()
        w2h = w2.detach().to(device=device, dtype=torch.float16).contiguous()
        b1f = b1.detach().to(device=device, dtype=torch.float32).contiguous() if b1 is not None else None
        self.b2 = b2.detach().to(device=device, dtype=torch.float32).contiguous() if b2 is not None else None
        nbytes = lib().sdk_ff_packed_bytes(Cc, self.features)
        self.packed = torch.empty(nbytes, dtype=torch.uint8, device=device)
        check(lib().sdk_ff_pack(_ptr(w1h), _ptr(b1f), _ptr(w2h), _ptr(self.packed), Cc, self.features, _stream()),
              "ff_pack")


def feed_forward(pf: PackedFF, t, residual=None, out=None):
    """out = residual + Linear2(GEGLU(t)) in one kernel (t, residual: [M, C] fp16 token rows)."""
    _need_cuda(t, "feed_forward t")
    M, Cc = t.shape
    if Cc != pf.channels or t.stride(-1) != 1:
        raise ValueError("sd_amd.feed_forward: t must be [M, channels] with unit column stride")
    if out is None:
        out = torch.empty(M, Cc, dtype=torch.float16, device=t.device)
    _claim(out)
    a = FfArgs()
    a.t, a.out, a.packed = t.data_ptr(), out.data_ptr(), pf.packed.data_ptr()
    a.b2 = pf.b2.data_ptr() if pf.b2 is not None else None
    if residual is not None:
        _need_cuda(residual, "feed_forward residual")
        a.res, a.res_ld = residual.data_ptr(), residual.stride(0)
    a.t_ld, a.out_ld = t.stride(0), out.stride(0)
    a.rows, a.channels, a.features = M, Cc, pf.features
    if PROFILER.active:
        PROFILER.begin("feed_forward", None, shape=(M, Cc, pf.features))
        PROFILER._cur = PROFILER._cur[:2] + (2.0 * M * Cc * 3 * pf.features,) + PROFILER._cur[3:]
    check(lib().sdk_feed_forward(C.byref(a), _stream()), "feed_forward")
    if PROFILER.active:
        PROFILER.end()
    return out


def token_linear_supported(in_features, out_features):
    return bool(lib().sdk_token_linear_supported(in_features, out_features))


class PackedTokenLinear:
    """A 320 -> 320 Linear / 1x1 conv for ``token_linear`` (sdk_token_linear): fp16 [out][in] weight
    (nn.Linear layout; a [out, in, 1, 1] conv weight is flattened), fp32 bias."""

    def __init__(self, w, b, device):
        w = w.detach().reshape(w.shape[0], -1)
        if not token_linear_supported(w.shape[1], w.shape[0]):
            raise ValueError(f"sd_amd.PackedTokenLinear: unsupported shape {tuple(w.shape)}")
        self.features = w.shape[0]
        self.w = w.to(device=device, dtype=torch.float16).contiguous()
        self.b = b.detach().to(device=device, dtype=torch.float32).contiguous() if b is not None else None


def token_linear(pk: PackedTokenLinear, x, residual=None, out=None, norm=None):
    """out = [residual +] x W^T + b (x, residual: [M, 320] fp16 token rows; out may be residual).
    ``norm=(gamma, beta, eps)`` (fp32 [320]) also returns LayerNorm(out) (sdk_token_linear_ln, the same
    bits as ``layer_norm(out, ...)``): ``(out, out_ln)``."""
    _need_cuda(x, "token_linear x")
    M, K = x.shape
    if K != pk.features or x.stride(-1) != 1:
        raise ValueError("sd_amd.token_linear: x must be [M, 320] with unit column stride")
    if out is None:
        out = torch.empty(M, pk.features, dtype=torch.float16, device=x.device)
    _claim(out)
    a = TokenLinearArgs()
    a.x, a.w, a.out = x.data_ptr(), pk.w.data_ptr(), out.data_ptr()
    a.bias = pk.b.data_ptr() if pk.b is not None else None
    if residual is not None:
        _need_cuda(residual, "token_linear residual")
        if residual.shape != (M, pk.features) or residual.stride(-1) != 1:
            raise ValueError("sd_amd.token_linear: residual must be [M, 320] with unit column stride")
        a.res, a.res_ld = residual.data_ptr(), residual.stride(0)
    a.x_ld, a.out_ld = x.stride(0), out.stride(0)
    a.rows, a.in_features, a.out_features = M, K, pk.features
    if PROFILER.active:
        PROFILER.begin("token_linear", None, shape=(M, pk.features, K))
        PROFILER._cur = PROFILER._cur[:2] + (2.0 * M * K * pk.features,) + PROFILER._cur[3:]
    if norm is None:
        check(lib().sdk_token_linear(C.byref(a), _stream()), "token_linear")
    else:
        g, bt, eps = norm
        _need_cuda(g, "token_linear_ln gamma", torch.float32)
        _need_cuda(bt, "token_linear_ln beta", torch.float32)
        if g.numel() != pk.features or bt.numel() != pk.features:
            raise ValueError("sd_amd.token_linear: norm gamma / beta must have 320 elements")
        out_ln = torch.empty(M, pk.features, dtype=torch.float16, device=x.device)
        check(lib().sdk_token_linear_ln(C.byref(a), g.data_ptr(), bt.data_ptr(), float(eps), out_ln.data_ptr(),
                                        out_ln.stride(0), _stream()), "token_linear_ln")
    if PROFILER.active:
        PROFILER.end()
    return out if norm is None else (out, out_ln)


# --------------------------------------------------------------------------- sampler glue

def token_embedding(ids: torch.Tensor, tok: torch.Tensor, pos: torch.Tensor):
    """CLIP token + position embedding: ids int64 [B, T] → fp16 [B, T, D] (fp32 tables)."""
    _need_cuda(ids, "token_embedding", torch.int64)
    _need_cuda(tok, "token_embedding table", torch.float32)
    _need_cuda(pos, "token_embedding positions", torch.float32)
    B, T = ids.shape
    if T > pos.shape[0]:
        raise ValueError(f"sd_amd.token_embedding: {T} tokens > {pos.shape[0]} positions")
    out = torch.empty(B, T, tok.shape[1], dtype=torch.float16, device=ids.device)
    check(lib().sdk_token_embedding(_ptr(ids.contiguous()), _ptr(tok), _ptr(pos), _ptr(out), B, T, tok.shape[1],
                                    _stream()), "token_embedding")
    return out


def extract_patches(z: torch.Tensor, kh: int, kw: int, sy: int, sx: int):
    """NCHW fp32 [B, C, H, W] → patches [Ly*Lx, B, C, kh, kw] (torch.nn.Unfold patch order)."""
    _need_cuda(z, "extract_patches", torch.float32)
    z = z.contiguous()
    B, Cc, H, W = z.shape
    Ly, Lx = (H - kh) // sy + 1, (W - kw) // sx + 1
    out = torch.empty(Ly * Lx, B, Cc, kh, kw, dtype=torch.float32, device=z.device)
    check(lib().sdk_extract_patches(_ptr(z), _ptr(out), B, Cc, H, W, kh, kw, sy, sx, _stream()), "extract_patches")
    return out


def fold_patches(patches: torch.Tensor, pix_w: torch.Tensor, l_w, H: int, W: int, sy: int, sx: int, Ly: int,
                 Lx: int):
    """[L, B, C, ph, pw] fp32 → normalised weighted overlap-add [B, C, H, W]."""
    _need_cuda(patches, "fold_patches", torch.float32)
    _need_cuda(pix_w, "fold_patches weights", torch.float32)
    patches = patches.contiguous()
    L, B, Cc, ph, pw = patches.shape
    assert L == Ly * Lx
    out = torch.empty(B, Cc, H, W, dtype=torch.float32, device=patches.device)
    check(lib().sdk_fold_patches(_ptr(patches), _ptr(pix_w.contiguous()), _ptr(l_w), _ptr(out), B, Cc, H, W, ph, pw,
                                 sy, sx, Ly, Lx, _stream()), "fold_patches")
    return out


def timestep_embedding(t: torch.Tensor, freqs: torch.Tensor, dim: int):
    _need_cuda(t, "timestep_embedding", torch.int64)
    out = torch.empty(t.shape[0], dim, dtype=torch.float16, device=t.device)
    check(lib().sdk_timestep_embedding(_ptr(t), _ptr(freqs), _ptr(out), t.shape[0], dim, _stream()),
          "timestep_embedding")
    return out


def nchw_to_nhwc(x: torch.Tensor, c_pad: int, scale: float = 1.0):
    _need_cuda(x, "nchw_to_nhwc", torch.float32)
    x = x.contiguous()
    B, Cc, H, W = x.shape
    y = torch.empty(B, H, W, c_pad, dtype=torch.float16, device=x.device)
    check(lib().sdk_nchw_to_nhwc(_ptr(x), _ptr(y), B, Cc, H * W, c_pad, C.c_float(scale), _stream()),
          "nchw_to_nhwc")
    return y


def ddim_step(x, e, sc: dict, noise=None, e_uncond=None, guidance=1.0, v_param=None, x_prev=None, pred_x0=None,
              temperature=1.0):
    """Fused DDIM update; ``sc`` holds the fp32 scalars (sampler.DDIMSampler computes them)."""
    _need_cuda(x, "ddim_step", torch.float32)
    _need_cuda(e, "ddim_step", torch.float32)
    x, e = x.contiguous(), e.contiguous()
    if e_uncond is not None:
        e_uncond = e_uncond.contiguous()
    if noise is not None:
        noise = noise.contiguous()
    a = DdimArgs()
    xp = x_prev if x_prev is not None else torch.empty_like(x)
    p0 = pred_x0 if pred_x0 is not None else torch.empty_like(x)
    a.x, a.e, a.x_prev, a.pred_x0 = x.data_ptr(), e.data_ptr(), xp.data_ptr(), p0.data_ptr()
    a.e_uncond = e_uncond.data_ptr() if e_uncond is not None else None
    a.noise = noise.data_ptr() if noise is not None else None
    a.n = x.numel()
    a.sqrt_one_minus_at = float(sc["sqrt_one_minus_at"])
    a.sqrt_at = float(sc["sqrt_at"])
    a.dir_coef = float(sc["dir_coef"])
    a.sqrt_a_prev = float(sc["sqrt_a_prev"])
    a.sigma = float(sc["sigma"])
    a.temperature = float(temperature)
    a.guidance = float(guidance)
    if v_param is not None:
        a.v_param = 1
        a.v_sqrt_a, a.v_sqrt_1ma = float(v_param[0]), float(v_param[1])
    check(lib().sdk_ddim_step(C.byref(a), _stream()), "ddim_step")
    return xp, p0


def diag_gaussian_sample(moments: torch.Tensor, noise=None, scale: float = 1.0, out=None):
    """moments NCHW fp32 [B, 2C, H, W] -> scale * (mean + std * noise) (or scale * mean) [B, C, H, W]."""
    _need_cuda(moments, "diag_gaussian_sample", torch.float32)
    B, C2, H, W = moments.shape
    moments = moments.contiguous()
    if noise is not None:
        _need_cuda(noise, "diag_gaussian_sample noise", torch.float32)
        noise = noise.contiguous()
    z = out if out is not None else torch.empty(B, C2 // 2, H, W, dtype=torch.float32, device=moments.device)
    check(lib().sdk_diag_gaussian_sample(_ptr(moments), _ptr(noise), _ptr(z), B, C2 // 2, H * W, float(scale),
                                         _stream()), "diag_gaussian_sample")
    return z


def stochastic_encode(x0: torch.Tensor, noise: torch.Tensor, sqrt_a: float, sqrt_1ma: float, out=None):
    """sqrt_a * x0 + sqrt_1ma * noise, fp32, bit-identical to the reference's CPU expression."""
    _need_cuda(x0, "stochastic_encode", torch.float32)
    _need_cuda(noise, "stochastic_encode noise", torch.float32)
    x0, noise = x0.contiguous(), noise.contiguous()
    y = out if out is not None else torch.empty_like(x0)
    check(lib().sdk_stochastic_encode(_ptr(x0), _ptr(noise), _ptr(y), x0.numel(), float(sqrt_a), float(sqrt_1ma),
                                      _stream()), "stochastic_encode")
    return y


def ddpm_step(x, eps, noise, inv_sqrt_alpha, coef, sigma, out=None):
    _need_cuda(x, "ddpm_step", torch.float32)
    y = out if out is not None else torch.empty_like(x)
    check(lib().sdk_ddpm_step(_ptr(x), _ptr(eps), _ptr(noise), _ptr(y), x.numel(), C.c_float(inv_sqrt_alpha),
                              C.c_float(coef), C.c_float(sigma), _stream()), "ddpm_step")
    return y


# --------------------------------------------------------------------------- profiling hooks

class _Profiler:
    """Optional per-launch HIP-event timing on the launch stream (bench roofline leg)."""

    def __init__(self):
        self.active = False
        self.records = []
        self.regions = []      # per record: the module region it ran in (None outside any)
        self.region = None     # set by modules around their launches (e.g. "cross_attention")
        self._cur = None

    def start(self):
        self.records = []
        self.regions = []
        self.active = True

    def stop(self):
        self.active = False

    def begin(self, kind, info, shape=None, nbytes=0):
        s = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        flops = info.flops if isinstance(info, ConvPlanInfo) else None
        if kind == "attention" and info is not None:
            b, h, nq, nk, d = info
            flops = 4.0 * b * h * nq * nk * d
            shape = info
        variant = info.variant if isinstance(info, ConvPlanInfo) else None
        self._cur = (kind, variant, flops, e0, shape, nbytes)

    def end(self):
        s = torch.cuda.current_stream()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(s)
        kind, variant, flops, e0, shape, nbytes = self._cur
        self.records.append((kind, variant, flops, e0, e1, shape, nbytes))
        self.regions.append(self.region)

    def region_summary(self, region):
        """Totals over the launches of one module region: launches, ms, flops, and per kind."""
        torch.cuda.synchronize()
        tot = {"launches": 0, "ms": 0.0, "flops": 0.0, "by_kind": {}}
        for rec, reg in zip(self.records, self.regions):
            if reg != region:
                continue
            kind, _, flops, e0, e1, _, _ = rec
            ms = e0.elapsed_time(e1)
            k = tot["by_kind"].setdefault(kind, {"launches": 0, "ms": 0.0, "flops": 0.0})
            for d in (tot, k):
                d["launches"] += 1
                d["ms"] += ms
                d["flops"] += flops or 0.0
        return tot

    def shape_table(self):
        """Per (kind, shape) totals: launches, ms, TFLOP/s — where the time goes."""
        torch.cuda.synchronize()
        out = {}
        for kind, variant, flops, e0, e1, shape, _ in self.records:
            d = out.setdefault((kind, shape), [0, 0.0, 0.0])
            d[0] += 1
            d[1] += e0.elapsed_time(e1)
            d[2] += flops or 0.0
        rows = [(k, v[0], v[1], (v[2] / (v[1] * 1e-3) / 1e12) if v[1] > 0 and v[2] else 0.0) for k, v in out.items()]
        return sorted(rows, key=lambda r: -r[2])

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for kind, variant, flops, e0, e1, shape, nbytes in self.records:
            key = kind if variant is None else f"{kind}:{variant}"
            d = out.setdefault(key, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["bytes"] += nbytes
            d["ms"] += e0.elapsed_time(e1)
            d["flops"] += flops or 0.0
        return out


PROFILER = _Profiler()
