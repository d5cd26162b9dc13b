"""ctypes bindings of libdcvc_hip (include/dcvc_hip.h) over PyTorch-ROCm memory.

Activations are ``Act`` views: a torch tensor ``buf`` of shape (H, W, Cbuf)
(NHWC, batch 1, on the GPU) plus a channel window (coff, C).  torch is only
the allocator and the stream provider; every computation below is one of our
kernels.  Calls are asynchronous on the current HIP stream.
"""
import ctypes
import os
import threading

import numpy as np
import torch

from ._native import NativeError, hip_lib, check

F32, BF16 = 0, 1
F16X3 = 2   # conv compute only: split-fp16 operands, fp32 views (dcvc_hip.h DCVC_F16X3)
ACT_NONE, ACT_LRELU, ACT_CLAMP01, ACT_ROUND = 0, 1, 2, 3
IN_NONE, IN_LRELU, IN_GATE = 0, 1, 2

_TORCH = {F32: torch.float32, BF16: torch.bfloat16}
_CNAME = {F32: "f32", BF16: "bf16", F16X3: "f16x3"}
_CODE = {torch.float32: F32, torch.bfloat16: BF16}


class CTensor(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("dtype", ctypes.c_int), ("H", ctypes.c_int),
                ("W", ctypes.c_int), ("C", ctypes.c_int), ("cstride", ctypes.c_int),
                ("coff", ctypes.c_int)]


class CDcbArgs(ctypes.Structure):
    _fields_ = [("x", CTensor), ("y", CTensor), ("cin", ctypes.c_int), ("cout", ctypes.c_int),
                ("gated", ctypes.c_int),
                ("w_conv1", ctypes.c_void_p), ("ld_conv1", ctypes.c_int), ("b_conv1", ctypes.c_void_p),
                ("w_dw", ctypes.c_void_p), ("b_dw", ctypes.c_void_p),
                ("w_conv2", ctypes.c_void_p), ("ld_conv2", ctypes.c_int), ("b_conv2", ctypes.c_void_p),
                ("w_adaptor", ctypes.c_void_p), ("ld_adaptor", ctypes.c_int), ("b_adaptor", ctypes.c_void_p),
                ("w_ffn1", ctypes.c_void_p), ("ld_ffn1", ctypes.c_int), ("b_ffn1", ctypes.c_void_p),
                ("w_ffn2", ctypes.c_void_p), ("ld_ffn2", ctypes.c_int), ("b_ffn2", ctypes.c_void_p),
                ("scale", ctypes.c_void_p), ("slope_dc", ctypes.c_float), ("slope_ffn", ctypes.c_float)]


class CConvArgs(ctypes.Structure):
    _fields_ = [("x", CTensor), ("y", CTensor), ("w", ctypes.c_void_p), ("bias", ctypes.c_void_p),
                ("cin", ctypes.c_int), ("cout", ctypes.c_int), ("kh", ctypes.c_int), ("kw", ctypes.c_int),
                ("stride", ctypes.c_int), ("pad", ctypes.c_int), ("compute", ctypes.c_int),
                ("in_op", ctypes.c_int), ("in_slope", ctypes.c_float), ("act", ctypes.c_int),
                ("slope", ctypes.c_float), ("shuffle", ctypes.c_int), ("scale", ctypes.c_void_p),
                ("res", CTensor), ("res2", CTensor)]


class CFfnArgs(ctypes.Structure):
    _fields_ = [("x", CTensor), ("y", CTensor), ("c", ctypes.c_int), ("hidden", ctypes.c_int),
                ("w", ctypes.c_void_p), ("b1", ctypes.c_void_p), ("b2", ctypes.c_void_p),
                ("scale", ctypes.c_void_p), ("slope", ctypes.c_float)]


class CDcArgs(ctypes.Structure):
    _fields_ = [("x", CTensor), ("y", CTensor), ("cin", ctypes.c_int), ("cout", ctypes.c_int),
                ("adaptor", ctypes.c_int), ("w", ctypes.c_void_p), ("b1", ctypes.c_void_p), ("wdw", ctypes.c_void_p),
                ("bdw", ctypes.c_void_p), ("b2", ctypes.c_void_p), ("ba", ctypes.c_void_p), ("slope", ctypes.c_float)]


class CDwcArgs(ctypes.Structure):
    _fields_ = [("t", CTensor), ("r", CTensor), ("y", CTensor), ("c", ctypes.c_int), ("w9", ctypes.c_void_p),
                ("bdw", ctypes.c_void_p), ("w2", ctypes.c_void_p), ("b2", ctypes.c_void_p)]


_T = CTensor
_vp, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
HIP_SYMBOLS = [
    ("dcvc_conv_pack_weights", ctypes.c_int64, [_vp, _i, _i, _i, _i, _i, _vp]),
    ("dcvc_conv2d", _i, [ctypes.POINTER(CConvArgs), _vp]),
    ("dcvc_set_option", _i, [ctypes.c_char_p, _i]),
    ("dcvc_split_range_flag", _i, [_vp]),
    ("dcvc_last_kernel", ctypes.c_char_p, []),
    ("dcvc_depthconv_block", _i, [ctypes.POINTER(CDcbArgs), _vp]),
    ("dcvc_ffn_pack_weights", ctypes.c_int64, [_vp, _vp, _i, _i, _vp]),
    ("dcvc_conv_ffn", _i, [ctypes.POINTER(CFfnArgs), _vp]),
    ("dcvc_dc_pack_weights", ctypes.c_int64, [_vp, _vp, _vp, _i, _i, _vp]),
    ("dcvc_depth_conv_split", _i, [ctypes.POINTER(CDcArgs), _vp]),
    ("dcvc_frag_pack_weights", ctypes.c_int64, [_vp, _i, _i, _vp]),
    ("dcvc_dw_conv2_split", _i, [ctypes.POINTER(CDwcArgs), _vp]),
    ("dcvc_dwconv3x3", _i, [_T, _T, _vp, _vp, _vp]),
    ("dcvc_flow_warp", _i, [_T, _T, _T, _vp, _vp, _vp]),
    ("dcvc_offset_diversity", _i, [_T, _T, _T, _T, _vp, _vp, _vp, _vp, _f, _vp]),
    ("dcvc_offset_diversity_workspace", ctypes.c_int64, [_i, _i]),
    ("dcvc_offset_diversity_ws", _i, [_T, _T, _T, _T, _vp, _vp, _vp, _vp, _f, _vp, ctypes.c_int64, _vp]),
    ("dcvc_resize2x", _i, [_T, _T, _i, _f, _vp]),
    ("dcvc_pool2x2", _i, [_T, _T, _i, _vp]),
    ("dcvc_add", _i, [_T, _T, _T, _vp]),
    ("dcvc_copy", _i, [_T, _T, _vp]),
    ("dcvc_pad_replicate", _i, [_T, _T, _vp]),
    ("dcvc_frame_to_nhwc", _i, [_vp, _i, _i, _T, _vp]),
    ("dcvc_frame_to_nhwc_zero_pad", _i, [_vp, _i, _i, _T, _vp]),
    ("dcvc_yuv420_to_nhwc", _i, [_vp, _vp, _i, _i, _T, _vp]),
    ("dcvc_frame_sse_workspace", ctypes.c_int64, []),
    ("dcvc_frame_sse", _i, [_T, _vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    ("dcvc_recon_to_u8", _i, [_T, _i, _i, _i, _vp, _vp]),
    ("dcvc_quadtree_encode_step", _i, [_T, _T, _T, _i, _T, _T, _vp, _vp, _f, _f, _vp]),
    ("dcvc_quadtree_indexes_step", _i, [_T, _T, _i, _vp, _f, _f, _vp]),
    ("dcvc_quadtree_decode_step", _i, [_T, _T, _i, _vp, _T, _T, _vp]),
    ("dcvc_nhwc_to_symbols", _i, [_T, _vp, _vp]),
    ("dcvc_symbols_to_nhwc", _i, [_vp, _T, _vp]),
    ("dcvc_quadtree_estimate_step", _i, [_T, _T, _T, _i, _T, _T, _vp, _i, _vp]),
    ("dcvc_factorized_bits", _i, [_T, _vp, _vp, _vp]),
    ("dcvc_sum_f32", _i, [_vp, ctypes.c_int64, _vp, _vp]),
    ("dcvc_dual_prior_encode_step", _i, [_T, _T, _T, _i, _T, _vp, _vp, _vp, _f, _f, _vp]),
    ("dcvc_dual_prior_indexes_step", _i, [_T, _T, _i, _vp, _f, _f, _vp]),
    ("dcvc_dual_prior_decode_step", _i, [_T, _T, _i, _vp, _T, _vp, _vp]),
    ("dcvc_dual_prior_estimate_step", _i, [_T, _T, _T, _i, _T, _vp, _vp, _i, _f, _vp]),
    ("dcvc_channel_div", _i, [_T, _vp, _T, _vp]),
    ("dcvc_fill", _i, [_T, _f, _vp]),
    ("dcvc_nhwc_to_symbols_i32", _i, [_T, _vp, _vp]),
    ("dcvc_symbols_i32_to_nhwc", _i, [_vp, _T, _vp]),
    ("dcvc_se_scale", _i, [_T, _vp, _vp, _i, _vp, _vp, _vp]),
    ("dcvc_se_apply", _i, [_T, _T, _vp, _T, _vp]),
    ("dcvc_yuv_planes_f64", _i, [_T, _vp, _vp, _i, _i, _vp, _vp, _vp]),
    ("dcvc_ssim_workspace", ctypes.c_int64, []),
    ("dcvc_ssim_level", _i, [_vp, _vp, _i, _i, _vp, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp]),
    ("dcvc_down2_f64", _i, [_vp, _i, _i, _vp, _vp]),
    ("dcvc_rgb_planes_f64", _i, [_T, _vp, _i, _i, _vp, _vp, _vp]),
    ("dcvc_avgpool2_f64", _i, [_vp, _i, _i, _vp, _vp]),
    ("dcvc_debug_poison_lds", _i, [_i, _i, _vp]),
    ("dcvc_debug_poison_vgpr", _i, [_i, _vp]),
]

_L = None

# Optional per-launch timing (bench.py roofline): when a list, each kernel
# wrapper records (family, start event, end event, algorithmic flops, bytes).
PROFILE = None


def _t0():
    if PROFILE is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _t1(e0, family, flops, nbytes, key=""):
    if e0 is None:
        return
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    PROFILE.append((family, e0, e, flops, nbytes, key))


def _esz(dtype):
    return 4 if dtype == F32 else 2


def lib():
    global _L
    if _L is None:
        _L = hip_lib()
        # DCVC_HIP_OPTIONS="name=v,name=v": dcvc_set_option switches applied at
        # load (whole-bench kernel A/B runs, e.g. "wconv=1"); unset in production
        for kv in filter(None, os.environ.get("DCVC_HIP_OPTIONS", "").split(",")):
            k, _, v = kv.partition("=")
            check(_L.dcvc_set_option(k.strip().encode(), int(v)), "set_option")
    return _L


def set_option(name, value):
    check(lib().dcvc_set_option(name.encode(), int(value)), "set_option")


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_get_device = getattr(torch._C, "_cuda_getDevice", None)


_tls = threading.local()

# Experiment switch (DCVC_BLOCKING_COPIES=1): host<->device symbol / index
# transfers as blocking copies instead of async copies on the stream.
ASYNC_COPIES = os.environ.get("DCVC_BLOCKING_COPIES", "0") != "1"


class SplitRangeError(NativeError):
    """A value entering a split-fp16 product was outside the split's range
    (|v| >= 2^15, dcvc_split_range_flag): the frame's result would not carry the
    ~2^-21 operand precision Precision.split() promises."""


def split_guard_arm(device):
    """Arm the fp16 range guard of the split kernels for the calling host
    thread (one device int32 flag per thread and device; the kernels launched
    from this thread raise it).  The flag is cleared (stream-ordered before
    the kernels it guards), so a value left by an earlier, unguarded call can
    never be charged to this one."""
    g = getattr(_tls, "split_flag", None)
    if g is None or g.device != device:
        g = torch.zeros(1, dtype=torch.int32, device=device)
        _tls.split_flag = g
    else:
        g.zero_()
    check(lib().dcvc_split_range_flag(g.data_ptr()), "split_range_flag")
    return g


def split_guard_disarm():
    """Stop the calling thread's split kernels from writing a flag (kernels
    launched outside a guarded call then write nothing; the pointer of a
    flag on another device is never left behind)."""
    check(lib().dcvc_split_range_flag(None), "split_range_flag")


def split_guard_tripped():
    """Whether a split kernel launched from this thread since the last arm
    saw |v| >= 2^15 (synchronises the current stream)."""
    g = getattr(_tls, "split_flag", None)
    return g is not None and bool(int(g.item()))


def split_guard_check(what="frame"):
    """Read and clear the calling thread's range flag (synchronises the current
    stream); raise SplitRangeError when a split kernel raised it."""
    g = getattr(_tls, "split_flag", None)
    if g is None:
        return
    if int(g.item()):
        g.zero_()
        raise SplitRangeError(f"{what}: a value entering a split-fp16 product had |v| >= 2^15, beyond the split's "
                              "range (hi + 2^-11 lo of fp16); code this input with Precision.parity()")


def pinned(key, n, dtype):
    """Persistent pinned host staging buffer of this host thread (first n
    elements).  Freeing a pinned tensor whose async H2D copy may still be in
    flight lets torch's process-wide pinned cache hand the block to another
    thread (another GOP lane) that overwrites it; buffers that live as long as
    the thread, reused only after a sync on the thread's stream, cannot race."""
    d = getattr(_tls, "pinned", None)
    if d is None:
        d = _tls.pinned = {}
    t = d.get((key, dtype))
    if t is None or t.numel() < n:
        if t is not None:
            torch.cuda.current_stream().synchronize()  # no copy of the old buffer in flight
        t = torch.empty(max(n, 1), dtype=dtype, pin_memory=True)
        d[(key, dtype)] = t
    return t[:n]


def upload(arr, device, key):
    """Host numpy array -> new device tensor, through this thread's pinned
    staging buffer for `key` (async H2D on the current stream).  A pageable
    source with non_blocking=True may be freed and reused by another host
    thread before the DMA reads it; a pinned staging buffer is rewritten only
    after its previous copy has completed (event per key)."""
    arr = np.ascontiguousarray(arr)
    d = getattr(_tls, "upload_ev", None)
    if d is None:
        d = _tls.upload_ev = {}
    ev = d.get(key)
    if ev is not None:
        ev.synchronize()
    dt = torch.from_numpy(arr.reshape(-1)[:0]).dtype
    src = pinned(("upload", key), arr.size, dt)
    src.numpy()[:] = arr.reshape(-1)
    out = torch.empty(arr.shape, dtype=dt, device=device)
    out.view(-1).copy_(src, non_blocking=ASYNC_COPIES)
    e = torch.cuda.Event()
    e.record()
    d[key] = e
    return out


def stream():
    """Raw handle of torch's current HIP stream on the current device.  The
    private torch._C accessors skip the Stream object torch.cuda.current_stream()
    builds (~8 us per launch, measured on the P-frame loop)."""
    if _raw_stream is not None and _get_device is not None:
        return _raw_stream(_get_device())
    return torch.cuda.current_stream().cuda_stream


class Act:
    """NHWC view: channels [coff, coff + C) of buf (H, W, Cbuf)."""
    __slots__ = ("buf", "coff", "C")

    def __init__(self, buf, coff=0, C=None):
        assert buf.dim() == 3 and buf.is_contiguous()
        self.buf = buf
        self.coff = coff
        self.C = buf.shape[2] - coff if C is None else C

    @property
    def H(self):
        return self.buf.shape[0]

    @property
    def W(self):
        return self.buf.shape[1]

    @property
    def dtype(self):
        return _CODE[self.buf.dtype]

    def ch(self, off, n):
        assert 0 <= off and off + n <= self.C
        return Act(self.buf, self.coff + off, n)

    def c(self):
        return CTensor(self.buf.data_ptr(), self.dtype, self.H, self.W, self.C, self.buf.shape[2], self.coff)

    def t(self):
        """torch view (H, W, C)."""
        return self.buf[:, :, self.coff:self.coff + self.C]

    def nchw(self):
        return self.t().permute(2, 0, 1).unsqueeze(0).float()

    def nchw_view(self):
        """(1, C, H, W) torch view of the same memory (no copy): what the
        reference harness receives as x_hat / dpb["ref_frame"]; in-place ops
        on it (test_video.py's clamp_) act on this buffer."""
        return self.t().permute(2, 0, 1).unsqueeze(0)


NULL_T = CTensor(None, 0, 0, 0, 0, 0, 0)


# Debug aid (DCVC_CANARY=1): every Act is allocated with a 4 KiB tail filled
# with a pattern; check_canaries() reports allocations whose tail a kernel
# overwrote (an out-of-bounds store).
CANARY = None
_CANARY_BYTES = 4096


# Debug aid (DCVC_POISON=nan|rand): every K.empty activation starts as NaN or
# as random bits (different per allocation) instead of whatever the caching
# allocator hands back, so a kernel that reads elements nobody wrote shows up
# as NaN or as an encoder/decoder divergence.
POISON = os.environ.get("DCVC_POISON", "")


def _poison(t):
    if POISON == "nan":
        t.view(torch.int16 if t.element_size() == 2 else torch.int32).fill_(-1)
    elif POISON == "rand":
        v = t.view(torch.int16 if t.element_size() == 2 else torch.int32)
        v.random_(-(1 << 15) if t.element_size() == 2 else -(1 << 31), (1 << 15) if t.element_size() == 2 else (1 << 31))
    return t


def _alloc(H, W, C, dtype, dev, zero):
    if CANARY is None:
        if zero:
            return Act(torch.zeros((H, W, C), dtype=_TORCH[dtype], device=dev))
        t = torch.empty((H, W, C), dtype=_TORCH[dtype], device=dev)
        return Act(_poison(t) if POISON else t)
    import traceback
    n = H * W * C
    es = 4 if dtype == F32 else 2
    flat = torch.empty(n * es + _CANARY_BYTES, dtype=torch.uint8, device=dev)
    flat[n * es:].fill_(0xA5)
    if zero:
        flat[:n * es].zero_()
    CANARY.append((flat, n * es, (H, W, C, dtype), "".join(traceback.format_stack(limit=6)[:-2])))
    return Act(flat[:n * es].view(_TORCH[dtype]).view(H, W, C))


def check_canaries():
    bad = []
    for flat, off, shape, where in CANARY or []:
        tail = flat[off:]
        if not bool((tail == 0xA5).all()):
            first = int((tail != 0xA5).nonzero()[0])
            bad.append((shape, first, where))
    return bad


def empty(H, W, C, dtype, device=None):
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return _alloc(H, W, C, dtype, dev, False)


def zeros(H, W, C, dtype, device=None):
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return _alloc(H, W, C, dtype, dev, True)


def from_nchw(x, dtype=F32):
    """(1, C, H, W) tensor -> Act (test / harness helper)."""
    t = x[0].permute(1, 2, 0).contiguous().to(_TORCH[dtype])
    if not t.is_cuda:
        t = t.cuda()
    return Act(t)


class ConvW:
    """A conv layer's packed weights.  Reference layout [Cout][Cin][kh][kw]
    (nn.Conv2d state_dict), packed once to [Cout][kh][kw][Cin_pad32]."""

    def __init__(self, weight, bias, stride=1, compute=BF16, device=None):
        w = weight.detach().float().cpu().contiguous()
        self.cout, self.cin, self.kh, self.kw = (int(s) for s in w.shape)
        self.stride = stride
        self.pad = (self.kh - 1) // 2
        self.compute = compute
        cinp = (self.cin + 31) // 32 * 32
        wn = w.numpy()
        if compute == F16X3:
            n = int(check(int(lib().dcvc_conv_pack_weights(wn.ctypes.data_as(ctypes.c_void_p), self.cout, self.cin,
                                                           self.kh, self.kw, compute, None)), "conv_pack_weights"))
        else:
            n = self.cout * self.kh * self.kw * cinp
        host = np.zeros(n, dtype=np.float32 if compute == F32 else np.uint16)
        got = lib().dcvc_conv_pack_weights(wn.ctypes.data_as(ctypes.c_void_p), self.cout, self.cin,
                                           self.kh, self.kw, compute, host.ctypes.data_as(ctypes.c_void_p))
        check(int(got), "conv_pack_weights")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if compute == F32:
            self.w = torch.from_numpy(host).to(dev)
        else:
            self.w = torch.from_numpy(host.view(np.int16)).to(dev)
        b = bias.detach().float().cpu() if bias is not None else torch.zeros(self.cout)
        self.b = b.contiguous().to(dev)

    def out_hw(self, H, W):
        return (H + 2 * self.pad - self.kh) // self.stride + 1, (W + 2 * self.pad - self.kw) // self.stride + 1


def conv(cw, x, y=None, *, out_dtype=None, in_op=IN_NONE, in_slope=0.0, act=ACT_NONE, slope=0.0,
         shuffle=False, scale=None, res=None, res2=None):
    """y = scale * (res2 + (res + act(conv(in_op(x)) + bias))), optional pixel shuffle."""
    Ho, Wo = cw.out_hw(x.H, x.W)
    cy = cw.cout // 4 if shuffle else cw.cout
    if y is None:
        f = 2 if shuffle else 1
        y = empty(Ho * f, Wo * f, cy, out_dtype if out_dtype is not None else x.dtype, x.buf.device)
    a = CConvArgs()
    a.x = x.c()
    a.y = y.c()
    a.w = cw.w.data_ptr()
    a.bias = cw.b.data_ptr()
    a.cin, a.cout, a.kh, a.kw = cw.cin, cw.cout, cw.kh, cw.kw
    a.stride, a.pad, a.compute = cw.stride, cw.pad, cw.compute
    a.in_op, a.in_slope, a.act, a.slope = in_op, in_slope, act, slope
    a.shuffle = 1 if shuffle else 0
    a.scale = scale.data_ptr() if scale is not None else None
    a.res = res.c() if res is not None else NULL_T
    a.res2 = res2.c() if res2 is not None else NULL_T
    e0 = _t0()
    check(lib().dcvc_conv2d(ctypes.byref(a), stream()), "conv2d")
    if e0 is not None:
        flops = 2 * Ho * Wo * cw.cout * cw.cin * cw.kh * cw.kw
        nb = (x.H * x.W * x.C * _esz(x.dtype) + cw.w.numel() * cw.w.element_size()
              + y.H * y.W * y.C * _esz(y.dtype) * (1 + (res is not None) + (res2 is not None)))
        kname = lib().dcvc_last_kernel().decode()
        _t1(e0, kname.split("<")[0], flops, nb, f"{kname} | k{cw.kh}s{cw.stride} {cw.cin}->{cw.cout} {x.H}x{x.W} "
            f"{_CNAME[cw.compute]} in{x.dtype}out{y.dtype}{' shuf' if shuffle else ''}")
    return y


UNSUPPORTED = -3


class FfnW:
    """A ConvFFN's weights packed for the fused split-fp16 kernel (sffn.hip):
    w1 = conv.0 [hidden][c][1][1], w2 = conv.2 [c][hidden][1][1]."""

    def __init__(self, w1, b1, w2, b2, device=None):
        w1 = w1.detach().float().cpu().reshape(w1.shape[0], -1).contiguous().numpy()
        w2 = w2.detach().float().cpu().reshape(w2.shape[0], -1).contiguous().numpy()
        self.hidden, self.c = w1.shape
        vp = ctypes.c_void_p
        n = int(lib().dcvc_ffn_pack_weights(w1.ctypes.data_as(vp), w2.ctypes.data_as(vp), self.c, self.hidden, None))
        check(n, "ffn_pack_weights")
        host = np.zeros(n, dtype=np.uint16)
        check(int(lib().dcvc_ffn_pack_weights(w1.ctypes.data_as(vp), w2.ctypes.data_as(vp), self.c, self.hidden,
                                               host.ctypes.data_as(vp))), "ffn_pack_weights")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.w = torch.from_numpy(host.view(np.int16)).to(dev)
        self.b1 = b1.detach().float().contiguous().to(dev)
        self.b2 = b2.detach().float().contiguous().to(dev)


class DcW:
    """A DepthConv's weights packed for the fused split-fp16 kernel (sdc.hip):
    conv1 [cin][cin], conv2 [cout][cin], adaptor [cout][cin] or None, the
    depthwise taps w9c [9][cin] (device) and the biases."""

    def __init__(self, w1, b1, w9c, bdw, w2, b2, wa=None, ba=None, device=None):
        f = lambda w: w.detach().float().cpu().reshape(w.shape[0], -1).contiguous().numpy()  # noqa: E731
        w1n, w2n = f(w1), f(w2)
        wan = f(wa) if wa is not None else None
        self.cin, self.cout = w1n.shape[0], w2n.shape[0]
        vp = ctypes.c_void_p
        pa = wan.ctypes.data_as(vp) if wan is not None else None
        n = int(lib().dcvc_dc_pack_weights(w1n.ctypes.data_as(vp), w2n.ctypes.data_as(vp), pa, self.cin, self.cout,
                                           None))
        check(n, "dc_pack_weights")
        host = np.zeros(n, dtype=np.uint16)
        check(int(lib().dcvc_dc_pack_weights(w1n.ctypes.data_as(vp), w2n.ctypes.data_as(vp), pa, self.cin,
                                             self.cout, host.ctypes.data_as(vp))), "dc_pack_weights")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.w = torch.from_numpy(host.view(np.int16)).to(dev)
        g = lambda t: t.detach().float().contiguous().to(dev)  # noqa: E731
        self.b1, self.w9c, self.bdw, self.b2 = g(b1), g(w9c), g(bdw), g(b2)
        self.ba = g(ba) if wa is not None else None


class DwcW:
    """The tail of a latent DepthConv packed for dcvc_dw_conv2_split: the
    depthwise taps w9c [9][c] (device) and bias, conv2 [c][c] as MFMA
    fragments (dcvc_frag_pack_weights) and its bias."""

    def __init__(self, w9c, bdw, w2, b2, device=None):
        w = w2.detach().float().cpu().reshape(w2.shape[0], -1).contiguous().numpy()
        self.c = int(w.shape[0])
        vp = ctypes.c_void_p
        n = int(check(int(lib().dcvc_frag_pack_weights(w.ctypes.data_as(vp), self.c, self.c, None)), "frag_pack"))
        host = np.zeros(n, dtype=np.uint16)
        check(int(lib().dcvc_frag_pack_weights(w.ctypes.data_as(vp), self.c, self.c, host.ctypes.data_as(vp))),
              "frag_pack")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.w2 = torch.from_numpy(host.view(np.int16)).to(dev)
        g = lambda t: t.detach().float().contiguous().to(dev)  # noqa: E731
        self.w9c, self.bdw, self.b2 = g(w9c), g(bdw), g(b2)


def dw_conv2_split(dwc, t, r, y=None):
    """y = conv2(dw3x3(t) + bdw) + b2 + r in one kernel (dcvc_dw_conv2_split);
    None when no kernel is instantiated for the width."""
    if y is None:
        y = empty(t.H, t.W, dwc.c, F32, t.buf.device)
    a = CDwcArgs()
    a.t, a.r, a.y, a.c = t.c(), r.c(), y.c(), dwc.c
    a.w9, a.bdw, a.w2, a.b2 = dwc.w9c.data_ptr(), dwc.bdw.data_ptr(), dwc.w2.data_ptr(), dwc.b2.data_ptr()
    e0 = _t0()
    rc = lib().dcvc_dw_conv2_split(ctypes.byref(a), stream())
    if rc == UNSUPPORTED:
        return None
    check(rc, "dw_conv2_split")
    if e0 is not None:
        n = t.H * t.W
        kname = lib().dcvc_last_kernel().decode()
        _t1(e0, kname.split("<")[0], 2 * n * dwc.c * (9 + dwc.c), n * dwc.c * 4 * 3 + dwc.w2.numel() * 2,
            f"{kname} | dw+conv2 {dwc.c} {t.H}x{t.W} f16x3")
    return y


def depth_conv_split(dw, x, y=None, slope=0.01):
    """DepthConv (conv1, LeakyReLU, depthwise 3x3, conv2, + identity) in one
    kernel (dcvc_depth_conv_split); None when not instantiated for the shape."""
    if y is None:
        y = empty(x.H, x.W, dw.cout, F32, x.buf.device)
    a = CDcArgs()
    a.x, a.y = x.c(), y.c()
    a.cin, a.cout, a.adaptor = dw.cin, dw.cout, 1 if dw.ba is not None else 0
    a.w, a.b1, a.wdw, a.bdw, a.b2 = dw.w.data_ptr(), dw.b1.data_ptr(), dw.w9c.data_ptr(), dw.bdw.data_ptr(), \
        dw.b2.data_ptr()
    a.ba = dw.ba.data_ptr() if dw.ba is not None else None
    a.slope = slope
    e0 = _t0()
    r = lib().dcvc_depth_conv_split(ctypes.byref(a), stream())
    if r == UNSUPPORTED:
        return None
    check(r, "depth_conv_split")
    if e0 is not None:
        n = x.H * x.W
        kname = lib().dcvc_last_kernel().decode()
        fl = 2 * n * (dw.cin * dw.cin + 9 * dw.cin + dw.cin * dw.cout * (2 if dw.ba is not None else 1))
        _t1(e0, kname.split("<")[0], fl, n * (dw.cin + dw.cout) * 4 + dw.w.numel() * 2,
            f"{kname} | depthconv {dw.cin}->{dw.cout} {x.H}x{x.W} f16x3")
    return y


def conv_ffn(fw, x, y=None, scale=None, slope=0.1):
    """y = scale * (x + lrelu(ffn2(lrelu(ffn1(x) + b1)) + b2)) in one kernel
    (dcvc_conv_ffn); None when no kernel is instantiated for the shape."""
    if y is None:
        y = empty(x.H, x.W, x.C, F32, x.buf.device)
    a = CFfnArgs()
    a.x, a.y = x.c(), y.c()
    a.c, a.hidden = fw.c, fw.hidden
    a.w, a.b1, a.b2 = fw.w.data_ptr(), fw.b1.data_ptr(), fw.b2.data_ptr()
    a.scale = scale.data_ptr() if scale is not None else None
    a.slope = slope
    e0 = _t0()
    r = lib().dcvc_conv_ffn(ctypes.byref(a), stream())
    if r == UNSUPPORTED:
        return None
    check(r, "conv_ffn")
    if e0 is not None:
        n = x.H * x.W
        kname = lib().dcvc_last_kernel().decode()
        _t1(e0, kname.split("<")[0], 4 * n * fw.c * fw.hidden, n * fw.c * 4 * 3 + fw.w.numel() * 2,
            f"{kname} | ffn {fw.c}->{fw.hidden}->{fw.c} {x.H}x{x.W} f16x3")
    return y


def depthconv_block(blk, x, y, scale=None):
    """Fused DepthConvBlock(2) (dcvc_depthconv_block).  Returns y, or None when
    no fused kernel is instantiated for this shape (caller runs unfused)."""
    a = CDcbArgs()
    a.x, a.y = x.c(), y.c()
    a.cin, a.cout, a.gated = blk.conv1.cin, blk.ffn2.cout, 1 if blk.gated else 0
    cp = lambda cw: (cw.w.data_ptr(), cw.w.numel() // cw.cout, cw.b.data_ptr())  # noqa: E731
    a.w_conv1, a.ld_conv1, a.b_conv1 = cp(blk.conv1)
    a.w_dw, a.b_dw = blk.dw[0].data_ptr(), blk.dw[1].data_ptr()
    a.w_conv2, a.ld_conv2, a.b_conv2 = cp(blk.conv2)
    if blk.adaptor is not None:
        a.w_adaptor, a.ld_adaptor, a.b_adaptor = cp(blk.adaptor)
    a.w_ffn1, a.ld_ffn1, a.b_ffn1 = cp(blk.ffn1)
    a.w_ffn2, a.ld_ffn2, a.b_ffn2 = cp(blk.ffn2)
    a.scale = scale.data_ptr() if scale is not None else None
    a.slope_dc, a.slope_ffn = blk.slope_dc, blk.slope_ffn
    e0 = _t0()
    r = lib().dcvc_depthconv_block(ctypes.byref(a), stream())
    if r == UNSUPPORTED:
        return None
    check(r, "depthconv_block")
    if e0 is not None:
        hid = 2 * a.cout if blk.gated else max(min(4 * a.cout, 1024), 2 * a.cout)
        n = x.H * x.W
        fl = 2 * n * (a.cin * a.cin + 9 * a.cin + a.cin * a.cout * (2 if blk.adaptor is not None else 1)
                      + a.cout * hid * (3 if blk.gated else 2))
        kname = lib().dcvc_last_kernel().decode()
        _t1(e0, kname.split("<")[0], fl, n * (a.cin + a.cout) * 2, f"{kname} | dcb {a.cin}->{a.cout} {x.H}x{x.W}")
    return y


def dwconv3x3(x, w9c, b, y=None):
    if y is None:
        y = empty(x.H, x.W, x.C, x.dtype, x.buf.device)
    e0 = _t0()
    check(lib().dcvc_dwconv3x3(x.c(), y.c(), w9c.data_ptr(), b.data_ptr(), stream()), "dwconv3x3")
    _t1(e0, "dwconv", 18 * x.H * x.W * x.C, x.H * x.W * x.C * (_esz(x.dtype) + _esz(y.dtype)),
        f"dwconv | {x.H}x{x.W}x{x.C}")
    return y


def flow_warp(x, flow, grid, y=None):
    if y is None:
        y = empty(x.H, x.W, x.C, x.dtype, x.buf.device)
    gx, gy = grid
    e0 = _t0()
    check(lib().dcvc_flow_warp(x.c(), flow.c(), y.c(), gx.data_ptr(), gy.data_ptr(), stream()), "flow_warp")
    _t1(e0, "warp", 8 * y.H * y.W * y.C, y.H * y.W * (y.C * (_esz(x.dtype) + _esz(y.dtype)) + 8),
        f"warp | {y.H}x{y.W}x{y.C}")
    return y


OD_PLANAR = False  # fp32 OffsetDiversity through the group-planar kernel pair (A/B switch)


def offset_diversity(feat, offs_half, flow, fw, fb, grid, y=None, max_mag=40.0):
    if y is None:
        y = empty(feat.H, feat.W, 48, feat.dtype, feat.buf.device)
    gx, gy = grid
    e0 = _t0()
    if feat.dtype == F32 and OD_PLANAR:
        # fp32 maps: the group-planar kernel pair, with a stream-ordered
        # workspace from torch's caching allocator (the feature's planar copy)
        n = int(lib().dcvc_offset_diversity_workspace(y.H, y.W))
        ws = torch.empty(n // 4, dtype=torch.float32, device=y.buf.device)
        check(lib().dcvc_offset_diversity_ws(feat.c(), offs_half.c(), flow.c(), y.c(), fw.data_ptr(), fb.data_ptr(),
                                             gx.data_ptr(), gy.data_ptr(), max_mag, ws.data_ptr(), n, stream()),
              "offset_diversity")
    else:
        check(lib().dcvc_offset_diversity(feat.c(), offs_half.c(), flow.c(), y.c(), fw.data_ptr(), fb.data_ptr(),
                                          gx.data_ptr(), gy.data_ptr(), max_mag, stream()), "offset_diversity")
    _t1(e0, "offset_diversity", y.H * y.W * 48 * 20, y.H * y.W * (96 * _esz(feat.dtype) + 8),
        f"offset_diversity | {y.H}x{y.W}")
    return y


def resize2x(x, up, mul=1.0, y=None, out_dtype=None):
    if y is None:
        H, W = (x.H * 2, x.W * 2) if up else (x.H // 2, x.W // 2)
        y = empty(H, W, x.C, out_dtype if out_dtype is not None else x.dtype, x.buf.device)
    check(lib().dcvc_resize2x(x.c(), y.c(), 1 if up else 0, mul, stream()), "resize2x")
    return y


def pool2x2(x, is_max, y=None):
    if y is None:
        y = empty(x.H // 2, x.W // 2, x.C, x.dtype, x.buf.device)
    check(lib().dcvc_pool2x2(x.c(), y.c(), 1 if is_max else 0, stream()), "pool2x2")
    return y


def add(a, b, y=None):
    if y is None:
        y = empty(a.H, a.W, a.C, a.dtype, a.buf.device)
    check(lib().dcvc_add(a.c(), b.c(), y.c(), stream()), "add")
    return y


def copy(x, y):
    check(lib().dcvc_copy(x.c(), y.c(), stream()), "copy")
    return y


def pad_replicate(x, y):
    check(lib().dcvc_pad_replicate(x.c(), y.c(), stream()), "pad_replicate")
    return y


def frame_to_nhwc(src_u8, h, w, y, zero_pad=False):
    if zero_pad:
        check(lib().dcvc_frame_to_nhwc_zero_pad(src_u8.data_ptr(), h, w, y.c(), stream()), "frame_to_nhwc_zero_pad")
    else:
        check(lib().dcvc_frame_to_nhwc(src_u8.data_ptr(), h, w, y.c(), stream()), "frame_to_nhwc")
    return y


def yuv420_to_nhwc(y_u8, uv_u8, h, w, out):
    """uint8 device planes Y (h*w) and U|V (2*(h/2)*(w/2)) -> padded NHWC
    YCbCr 4:4:4 fp32 (ycbcr420_to_444(order=0) + pad, test_video.py:111-132)."""
    assert y_u8.dtype == torch.uint8 and uv_u8.dtype == torch.uint8
    assert y_u8.numel() == h * w and uv_u8.numel() == 2 * (h // 2) * (w // 2)
    check(lib().dcvc_yuv420_to_nhwc(y_u8.data_ptr(), uv_u8.data_ptr(), h, w, out.c(), stream()), "yuv420_to_nhwc")
    return out


def frame_sse_workspace(device):
    n = int(lib().dcvc_frame_sse_workspace())
    return torch.empty(n // 8, dtype=torch.float64, device=device)


def frame_sse(x_hat, src_u8, h, w, workspace, out3, uv_u8=None):
    """Clamp x_hat in place and write the 3 per-plane squared-error sums of
    the h x w crop into out3 (fp64 device); see dcvc_frame_sse."""
    assert x_hat.dtype == F32 and x_hat.C == 3 and out3.dtype == torch.float64 and out3.numel() >= 3
    yuv = uv_u8 is not None
    assert src_u8.numel() == (h * w if yuv else 3 * h * w)
    check(lib().dcvc_frame_sse(x_hat.c(), src_u8.data_ptr(), uv_u8.data_ptr() if yuv else None, h, w, int(yuv),
                               workspace.data_ptr(), out3.data_ptr(), stream()), "frame_sse")
    return out3


def recon_to_u8(x_hat, h, w, yuv420, out):
    """Decoded frame -> uint8 as the --save_decoded_frame writers store it
    (dcvc_recon_to_u8): HWC RGB, or Y | U | V planes."""
    n = h * w + 2 * (h // 2) * (w // 2) if yuv420 else 3 * h * w
    assert out.dtype == torch.uint8 and out.numel() >= n and x_hat.dtype == F32 and x_hat.C == 3
    check(lib().dcvc_recon_to_u8(x_hat.c(), h, w, 1 if yuv420 else 0, out.data_ptr(), stream()), "recon_to_u8")
    return out


def yuv_planes_f64(x_hat, y_u8, uv_u8, h, w, src, rec):
    """fp64 source / recon planes [Y | U | V] of the crop (calc_msssim's inputs)."""
    n = h * w + 2 * (h // 2) * (w // 2)
    assert src.dtype == torch.float64 and rec.dtype == torch.float64 and src.numel() >= n and rec.numel() >= n
    check(lib().dcvc_yuv_planes_f64(x_hat.c(), y_u8.data_ptr(), uv_u8.data_ptr(), h, w, src.data_ptr(),
                                    rec.data_ptr(), stream()), "yuv_planes_f64")


def ssim_level(a, b, h, w, window, workspace, out2):
    """Means of calc_ssim's ssim and cs maps of two fp64 h x w planes."""
    check(lib().dcvc_ssim_level(a.data_ptr(), b.data_ptr(), h, w, window.data_ptr(), 1e-4, 9e-4,
                                workspace.data_ptr(), out2.data_ptr(), stream()), "ssim_level")


def rgb_planes_f64(x_hat, src_u8, h, w, src, rec):
    assert src.numel() >= 3 * h * w and rec.numel() >= 3 * h * w
    check(lib().dcvc_rgb_planes_f64(x_hat.c(), src_u8.data_ptr(), h, w, src.data_ptr(), rec.data_ptr(), stream()),
          "rgb_planes_f64")


def avgpool2_f64(x, h, w, y):
    check(lib().dcvc_avgpool2_f64(x.data_ptr(), h, w, y.data_ptr(), stream()), "avgpool2_f64")


def down2_f64(x, h, w, y):
    check(lib().dcvc_down2_f64(x.data_ptr(), h, w, y.data_ptr(), stream()), "down2_f64")


def qt_encode_step(y, params, sm, k, yhs, yhat, sym, idx, log_min, log_step):
    check(lib().dcvc_quadtree_encode_step(y.c(), params.c(), sm.c() if sm is not None else NULL_T, k,
                                          yhs.c(), yhat.c(), sym.data_ptr(), idx.data_ptr(),
                                          log_min, log_step, stream()), "quadtree_encode_step")


def qt_indexes_step(params, sm, k, idx, log_min, log_step):
    check(lib().dcvc_quadtree_indexes_step(params.c(), sm.c() if sm is not None else NULL_T, k,
                                           idx.data_ptr(), log_min, log_step, stream()), "quadtree_indexes_step")


def qt_decode_step(params, sm, k, sym, yhs, yhat):
    check(lib().dcvc_quadtree_decode_step(params.c(), sm.c() if sm is not None else NULL_T, k,
                                          sym.data_ptr(), yhs.c(), yhat.c(), stream()), "quadtree_decode_step")


def to_symbols(x, sym):
    check(lib().dcvc_nhwc_to_symbols(x.c(), sym.data_ptr(), stream()), "nhwc_to_symbols")


def from_symbols(sym, y):
    check(lib().dcvc_symbols_to_nhwc(sym.data_ptr(), y.c(), stream()), "symbols_to_nhwc")


def qt_estimate_step(y, params, sm, k, yhs, yhat, bits, gaussian):
    check(lib().dcvc_quadtree_estimate_step(y.c(), params.c(), sm.c() if sm is not None else NULL_T, k,
                                            yhs.c(), yhat.c(), bits.data_ptr(), 1 if gaussian else 0, stream()),
          "quadtree_estimate_step")


def factorized_bits(z, table, bits):
    check(lib().dcvc_factorized_bits(z.c(), table.data_ptr(), bits.data_ptr(), stream()), "factorized_bits")


def sum_f32(x, out):
    """out (1-element fp32 device tensor) = fixed-order sum of x (fp32 device tensor)."""
    check(lib().dcvc_sum_f32(x.data_ptr(), x.numel(), out.data_ptr(), stream()), "sum_f32")
    return out


# ---- DCVC-HEM (hem.hip)
def _ptr(t):
    return t.data_ptr() if t is not None else None


def dp_encode_step(y, buf, sm, k, yhat, post, sym, idx, log_min, log_step):
    check(lib().dcvc_dual_prior_encode_step(y.c(), buf.c(), sm.c() if sm is not None else NULL_T, k, yhat.c(),
                                            _ptr(post), sym.data_ptr(), idx.data_ptr(), log_min, log_step,
                                            stream()), "dual_prior_encode_step")


def dp_indexes_step(buf, sm, k, idx, log_min, log_step):
    check(lib().dcvc_dual_prior_indexes_step(buf.c(), sm.c() if sm is not None else NULL_T, k, idx.data_ptr(),
                                             log_min, log_step, stream()), "dual_prior_indexes_step")


def dp_decode_step(buf, sm, k, sym, yhat, post):
    check(lib().dcvc_dual_prior_decode_step(buf.c(), sm.c() if sm is not None else NULL_T, k, sym.data_ptr(),
                                            yhat.c(), _ptr(post), stream()), "dual_prior_decode_step")


def dp_estimate_step(y, buf, sm, k, yhat, post, bits, gaussian, scale_min):
    check(lib().dcvc_dual_prior_estimate_step(y.c(), buf.c(), sm.c() if sm is not None else NULL_T, k, yhat.c(),
                                              _ptr(post), bits.data_ptr(), 1 if gaussian else 0, scale_min,
                                              stream()), "dual_prior_estimate_step")


def channel_div(x, q, y=None):
    if y is None:
        y = empty(x.H, x.W, x.C, F32, x.buf.device)
    check(lib().dcvc_channel_div(x.c(), q.data_ptr(), y.c(), stream()), "channel_div")
    return y


def to_symbols_i32(x, sym):
    check(lib().dcvc_nhwc_to_symbols_i32(x.c(), sym.data_ptr(), stream()), "nhwc_to_symbols_i32")


def from_symbols_i32(sym, y):
    check(lib().dcvc_symbols_i32_to_nhwc(sym.data_ptr(), y.c(), stream()), "symbols_i32_to_nhwc")


def se_scale(x, w1, w2, work, out):
    check(lib().dcvc_se_scale(x.c(), w1.data_ptr(), w2.data_ptr(), w1.shape[0], work.data_ptr(), out.data_ptr(),
                              stream()), "se_scale")
    return out


def se_apply(a, x, scale, y=None):
    if y is None:
        y = empty(a.H, a.W, a.C, a.dtype, a.buf.device)
    check(lib().dcvc_se_apply(a.c(), x.c(), scale.data_ptr(), y.c(), stream()), "se_apply")
    return y


def fill(y, value=0.0):
    check(lib().dcvc_fill(y.c(), float(value), stream()), "fill")
    return y
