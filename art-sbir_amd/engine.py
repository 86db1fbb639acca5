"""Executor of the ModifiedResNet hot path on libartsbir_hip (MI355X / gfx950).

The reference runs the encoder as a chain of PyTorch eager ops
(models.py:344-360: stem -> layer1..4 -> attnpool; Bottleneck.forward
models.py:223-236; AttentionPool2d.forward models.py:249-272) and lets
autograd record the backward.  Here the whole encoder forward and backward are
sequenced explicitly over the C-ABI kernels:

  * activations live in HBM as NHWC tensors of the compute dtype (bf16 for
    throughput, f32 for parity); the raw convolution outputs y are stored and
    BatchNorm+ReLU(+AvgPool) is applied once (act_pool / block_out), producing
    the next convolution's input, which is also the weight-gradient operand;
  * BN batch statistics come out of the convolution epilogue (sum / sum of
    squares) and are finalised per call -> per-branch statistics exactly as the
    reference's three separate forward calls (train.py:28-30);
  * several forward calls can run as one batch of G SEGMENTS (the triplet's
    sketch / positive / negative, ModifiedResNet.forward_branches): every
    GEMM runs once over G x B images, while BatchNorm statistics, running
    statistics and the BN backward stay per segment — the same arithmetic as G
    separate calls;
  * the BatchNorm backward reduction (sum g, sum g*xhat) of a BN whose output
    gradient comes out of a data-gradient GEMM is fused into that GEMM's
    epilogue (artsbir_conv2d_dgrad_bnb), which stores g = d * relu-mask;
  * weights are re-packed from the f32 parameters (reference layout, so
    state_dicts interchange) into the kernel layouts whenever a parameter
    changes (torch version counter or an optimizer step of optim.Adam here).

No op of this module runs on the CPU or through a PyTorch kernel except
allocation (torch.empty / torch.zeros) — the product path fails if the
native library is missing.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch

import _hip
from _hip import call, ptr

NSLOT = _hip.NSLOT
BN_EPS = 1e-5
BN_MOMENTUM = 0.1
# ARTSBIR_FUSE_BNB=0 runs the BN-backward reduction as its own pass (A/B tests)
FUSE_BNB = os.environ.get("ARTSBIR_FUSE_BNB", "1") != "0"
# ARTSBIR_OVERLAP_WGRAD=0 keeps the weight gradients on the caller's stream
OVERLAP_WGRAD = os.environ.get("ARTSBIR_OVERLAP_WGRAD", "1") != "0"
# ARTSBIR_WGRAD_MAIN=1x1 | 3x3: that class of weight gradients runs in order on
# the main stream instead of the side stream (experiment: HBM-bound 1x1 wgrads
# beside an HBM-bound main chain contend for bandwidth without hiding anything)
WGRAD_MAIN = os.environ.get("ARTSBIR_WGRAD_MAIN", "")
# ARTSBIR_MASK_BITS=0 makes the fused backward re-read the block output for its
# ReLU mask instead of the bit mask written by the forward
MASK_BITS = os.environ.get("ARTSBIR_MASK_BITS", "1") != "0"
# inference (eval BatchNorm, no autograd): every BatchNorm folded into its conv
# (artsbir_bn_fold) and applied with the ReLU / residual add in the conv's
# epilogue (artsbir_conv2d_fwd_act): no separate BN / activation passes.
# ARTSBIR_FUSED_EVAL=0 runs inference through the training-path kernels.
FUSED_EVAL = os.environ.get("ARTSBIR_FUSED_EVAL", "1") != "0"
# ARTSBIR_DETERMINISTIC=1 (parity runs): forward BatchNorm statistics
# by a fixed-order f64 reduction of the stored conv output (artsbir_bn_stats_det)
# instead of the epilogue's f32 atomics, so a forward is bit-identical from run
# to run and ReLU masks cannot flip between runs
DETERMINISTIC = os.environ.get("ARTSBIR_DETERMINISTIC", "0") == "1"
# ARTSBIR_FOLD_BN=0 runs the block-output BatchNorm backward (bn3 and the
# downsample BN) as its own apply pass before the 1x1 convs' data / weight
# gradients instead of folding it through them (artsbir_conv1x1_dgrad_fold)
FOLD_BN = [os.environ.get("ARTSBIR_FOLD_BN", "1") != "0"]
# the layer-1 fold data gradients also accumulate their weight-gradient operands
# (artsbir_conv1x1_dgrad_fold_wg): g and x read once for both gradients
FOLD_WG = [os.environ.get("ARTSBIR_FOLD_WG", "1") != "0"]
# ARTSBIR_FOLD_BN1=1 folds bn1's backward (models.py:199, conv1 -> bn1 of every
# Bottleneck) through conv1 with bn1's input y1 (the y-side fold,
# artsbir_conv1x1_dgrad_fold_y): dy1 is never written or read.  Off by default:
# its weight gradient needs g1^T x and y1^T x (twice conv1's weight-gradient
# MFMA work on the side stream), which cost the C2 step more than the apply
# pass it removes from the main stream (94.8 vs 91.2 ms on one box)
FOLD_BN1 = [os.environ.get("ARTSBIR_FOLD_BN1", "0") == "1"]


def set_deterministic(on: bool = True) -> bool:
    """switch the deterministic mode (fixed-order f64 BatchNorm reductions, forward
    and backward; unfused data gradients); returns the old value"""
    global DETERMINISTIC
    old, DETERMINISTIC = DETERMINISTIC, bool(on)
    _hip.lib().artsbir_set_deterministic(1 if DETERMINISTIC else 0)
    return old


# ARTSBIR_SIDE_CUS=K: the weight-gradient stream is restricted to K CUs (0: all)
SIDE_CUS = [int(os.environ.get("ARTSBIR_SIDE_CUS", "0"))]
SIDE_CONTIGUOUS = [False]  # measurement switch: those K CUs are mask bits 0..K-1
# ARTSBIR_WGRAD_DEFER=3x3|1x1|all: the side stream starts a layer's weight gradient
# only after that layer's data gradient has run on the main stream (instead of
# beside it), so the two GEMMs of one layer never compete for the same CUs
WGRAD_DEFER = [os.environ.get("ARTSBIR_WGRAD_DEFER", "")]
# the stem conv's weight gradient on the main stream (ARTSBIR_STEM_WGRAD_MAIN=0:
# on the side stream like the others)
STEM_WGRAD_MAIN = os.environ.get("ARTSBIR_STEM_WGRAD_MAIN", "1") != "0"
# measurement switch (never set in a real step): leave the weight gradients out
SKIP_WGRAD = [False]
_MASKED_STREAMS = {}


def cu_masked_stream(device, ncu, invert=False, contiguous=False):
    """a torch stream over a hipExtStreamCreateWithCUMask stream using ncu CUs
    spread evenly over the device's CUs (contiguous: mask bits 0..ncu-1), or
    (invert) every CU but those (cached per (device, ncu, invert, contiguous))"""
    key = (device.index if device.index is not None else 0, ncu, invert, contiguous)
    st = _MASKED_STREAMS.get(key)
    if st is not None:
        return st
    total = torch.cuda.get_device_properties(device).multi_processor_count
    ncu = max(1, min(ncu, total))
    words = (total + 31) // 32
    mask = (ctypes.c_uint * words)()
    for i in range(ncu):
        cu = i if contiguous else (i * total) // ncu
        mask[cu // 32] |= 1 << (cu % 32)
    if invert:
        for w in range(words):
            bits = min(32, total - 32 * w)
            mask[w] = ~mask[w] & ((1 << bits) - 1)
    handle = ctypes.c_void_p()
    with torch.cuda.device(device):
        call("artsbir_stream_create_cu_mask", mask, words, ctypes.byref(handle))
    st = torch.cuda.ExternalStream(handle.value, device=device)
    _MASKED_STREAMS[key] = st
    return st


PACK_EPB, PACK_T = 1024, 64  # artsbir_pack_weights blocking (PACK_EPB, PACK_T in elementwise.hip)


def _fuse_bnb():
    """BN-backward reductions fused into the data-gradient epilogues (f32 atomics)
    except in the deterministic mode, which reduces them in a fixed order"""
    return FUSE_BNB and not DETERMINISTIC

# bumped by optim.Adam (which updates parameters through raw pointers, invisible
# to torch's version counters) so packed weights are rebuilt after every step
WEIGHTS_GENERATION = [0]


def bump_weights_generation():
    WEIGHTS_GENERATION[0] += 1


def _s():
    return _hip.stream()


def _at(t, i):
    """raw pointer of image i of an NHWC tensor (None -> NULL)"""
    return None if t is None else t[i].data_ptr()


@dataclass
class BNState:
    """per-call batch-norm parameters of G segments: buf [G][4][C] f32 holds each
    segment's parameter block mean, istd, scale = gamma*istd, beta — applied by
    the kernels as (y - mean) * scale + beta; count = elements per segment."""
    buf: torch.Tensor
    count: float

    @property
    def G(self):
        return self.buf.shape[0]

    def seg(self, i):
        return BNState(self.buf[i:i + 1], self.count)

    @property
    def pstride(self):
        """floats between the parameters of consecutive segments"""
        return 4 * self.buf.shape[2]

    @property
    def mean(self):
        return self.buf[0, 0]

    @property
    def istd(self):
        return self.buf[0, 1]

    @property
    def scale(self):
        return self.buf[0, 2]

    @property
    def block(self):
        """the first segment's [4][C] parameter block (segments follow at 4*C floats)"""
        return self.buf[0]


@dataclass
class Act:
    """an NHWC activation tensor [B][H][W][C] and the affine(+ReLU) that must be
    applied when it is read (None: read as is)."""
    t: torch.Tensor
    bn: BNState | None = None
    relu: int = 0

    @property
    def shape(self):
        return tuple(self.t.shape)


class Engine:
    """Owns the packed weights of one ModifiedResNet and runs it on the GPU."""

    def __init__(self, model):
        self.model = model
        self._packed = None
        self._packed_key = None
        self.dtype = torch.float32
        self._G = 1
        # ddp.OverlappedReducer (or None): told which gradient ranges are final
        # as the backward proceeds, so the data-parallel all-reduce overlaps it
        self.grad_hook = None
        self._side_keep = []  # tensors the weight-gradient stream still reads (released at the join)
        self._eval = None      # folded conv weights + biases of the eval forward
        self._eval_key = None
        # bumped whenever a train-mode forward updates the BN running statistics
        # (artsbir_bn_finalize_seg writes them through raw pointers, invisible to
        # torch's version counters), so the folded eval weights are rebuilt
        self._bn_gen = 0

    # ------------------------------------------------------------------ utils
    @property
    def dt(self):
        return _hip.dtype_code(self.dtype)

    def _empty(self, *shape, dtype=None, device=None):
        return torch.empty(*shape, dtype=dtype or self.dtype, device=device)

    def _desc(self, N, H, W, C, Cout, R, S, stride, pad):
        return _hip.conv_desc(self.dtype, N, H, W, C, Cout, R, S, stride, pad)

    # ---------------------------------------------------------- weight packing
    def _params_key(self):
        return (self.dtype, WEIGHTS_GENERATION[0],
                tuple((p.data_ptr(), p._version) for p in self.model.parameters()))

    def packed(self):
        """packed operands of the current weights.  The first pack of a set of
        parameter storages allocates the buffers and records every pack; each
        later re-pack (after an optimizer step) rewrites the same buffers with
        ONE batched launch (artsbir_pack_weights) instead of ~120 small ones."""
        key = self._params_key()
        if self._packed_key != key:
            plan_key = (self.dtype, self.dt,
                        tuple((p.data_ptr(), tuple(p.shape), p.dtype) for p in self.model.parameters()))
            plan = getattr(self, "_plan", None)
            if plan is not None and plan[0] == plan_key and plan[4] == self._packed_ranges():
                call("artsbir_pack_weights", self.dt, ptr(plan[1]), plan[2], plan[3], _s(),
                     kernel="pack_weights_kernel", tag=f"pack_weights x{plan[2]}")
            else:
                self._recording = []
                self._packed = self._pack_all()
                self._plan = self._make_plan(plan_key, self._recording)
                self._recording = None
            self._packed_key = key
        return self._packed

    def _packed_ranges(self):
        """(data_ptr, nbytes) of every packed buffer the replay writes into"""
        out = []

        def walk(v):
            if isinstance(v, torch.Tensor):
                out.append((v.data_ptr(), v.numel() * v.element_size()))
            elif isinstance(v, (list, tuple)):
                for x in v:
                    walk(x)
            elif isinstance(v, dict):
                for x in v.values():
                    walk(x)
        walk(getattr(self, "_packed", None))
        return tuple(sorted(out))

    def _make_plan(self, plan_key, recs):
        if not recs:
            return None
        # the replay rewrites exactly the buffers _pack_all filled: every recorded
        # destination lies in a packed buffer, and every packed buffer was written
        # through a recorded pack (a pack added without recording would go stale)
        ranges = self._packed_ranges()
        hit = [False] * len(ranges)
        for rec in recs:
            dst = rec[1]
            inside = [i for i, (b, n) in enumerate(ranges) if b <= dst < b + n]
            assert inside, "re-pack plan: a recorded destination outside the packed buffers"
            for i in inside:
                hit[i] = True
        assert all(hit), "re-pack plan: a packed buffer written without a recorded pack"
        dev = next(self.model.parameters()).device
        descs = (_hip.PackDesc * len(recs))()
        blk = 0
        for d, (src, dst, co, ci, r, s, ci_pad, mode, ldo) in zip(descs, recs):
            d.src, d.dst, d.Co, d.Ci, d.R, d.S, d.ci_pad, d.mode, d.ldo, d.blk0 = \
                src, dst, co, ci, r, s, ci_pad, mode, ldo, blk
            if mode == 1:  # 64 x 64 tiles of the flipped transpose
                blk += -(-co // PACK_T) * -(-(ci * r * s) // PACK_T)
            else:
                blk += -(-(co * r * s * ci_pad if mode == 0 else co) // PACK_EPB)
        raw = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8)
        return (plan_key, raw.to(dev), len(recs), blk, ranges)

    def _pack_one(self, src, co, ci, r, s, ci_pad, mode, ldo, dst):
        call("artsbir_pack_weight", self.dt, ptr(src), co, ci, r, s, ci_pad, mode, ldo, ptr(dst), _s())
        if getattr(self, "_recording", None) is not None:
            self._recording.append((ptr(src), ptr(dst), co, ci, r, s, ci_pad, mode, ldo if ldo > 0 else co))

    def _pack_conv(self, conv, ci_pad=None, need_dgrad=True):
        w = conv.weight.detach()
        co, ci, r, s = w.shape
        ci_pad = ci_pad or ci
        fw = self._empty(co, r, s, ci_pad, device=w.device)
        self._pack_one(w, co, ci, r, s, ci_pad, 0, 0, fw)
        dw = None
        if need_dgrad:
            dw = self._empty(ci, r, s, co, device=w.device)
            self._pack_one(w, co, ci, r, s, ci, 1, co, dw)
        return fw, dw

    def _pack_linear_pair(self, lins, device):
        """rows-concatenated forward weight [sum out][in] and its transpose [in][sum out]"""
        outs = [l.weight.shape[0] for l in lins]
        fin = lins[0].weight.shape[1]
        tot = sum(outs)
        fw = self._empty(tot, fin, device=device)
        tw = self._empty(fin, tot, device=device)
        bias = torch.empty(tot, dtype=torch.float32, device=device)
        off = 0
        for l, o in zip(lins, outs):
            w = l.weight.detach()
            self._pack_one(w, o, fin, 1, 1, fin, 0, 0, fw[off:])
            self._pack_one(w, o, fin, 1, 1, fin, 1, tot, tw[:, off:])
            call("artsbir_cast", _hip.DT_F32, ptr(l.bias.detach()), _hip.DT_F32, ptr(bias[off:]), o, _s())
            if getattr(self, "_recording", None) is not None:  # mode 2: the bias copy
                self._recording.append((ptr(l.bias), ptr(bias[off:]), o, 1, 1, 1, 1, 2, o))
            off += o
        return fw, tw, bias

    def _pack_all(self):
        m = self.model
        dev = m.conv1.weight.device
        pk = {}
        pk["stem"] = [self._pack_conv(m.conv1, ci_pad=8, need_dgrad=False),
                      self._pack_conv(m.conv2), self._pack_conv(m.conv3)]
        blocks = []
        for blk in m.blocks():
            d = {"conv1": self._pack_conv(blk.conv1), "conv2": self._pack_conv(blk.conv2),
                 "conv3": self._pack_conv(blk.conv3)}
            if blk.downsample is not None:
                d["down"] = self._pack_conv(blk.downsample[1])
            blocks.append(d)
        pk["blocks"] = blocks
        ap = m.attnpool
        pk["kv"] = self._pack_linear_pair([ap.k_proj, ap.v_proj], dev)
        pk["q"] = self._pack_linear_pair([ap.q_proj], dev)
        pk["c"] = self._pack_linear_pair([ap.c_proj], dev)
        return pk

    # ------------------------------------------------------------- primitives
    def _gemm_nt(self, M, N, K, a, lda, b, c, ldc, out_f32, acc, bias):
        call("artsbir_gemm_nt", self.dt, M, N, K, ptr(a), lda, ptr(b), ptr(c), ldc, out_f32, acc, ptr(bias), None,
             _s(), kernel="auto", flops=2.0 * M * N * K, tag=f"gemm_nt {M}x{N}x{K} f32{out_f32} acc{acc}")

    def _gemm_tn(self, M, N, K, dy, ldd, x, ldx, dw):
        call("artsbir_gemm_tn", self.dt, M, N, K, ptr(dy), ldd, ptr(x), ldx, ptr(dw), _s(),
             kernel="auto", flops=2.0 * M * N * K, tag=f"gemm_tn {M}x{N}x{K}")

    def _side_gemm_tn(self, M, N, K, dy, ldd, x, ldx, dw):
        """_gemm_tn of a weight gradient on the side stream (as _wgrad), its
        operands held until the backward's stream join"""
        if not OVERLAP_WGRAD or SKIP_WGRAD[0]:
            if not SKIP_WGRAD[0]:
                self._gemm_tn(M, N, K, dy, ldd, x, ldx, dw)
            return
        main = torch.cuda.current_stream()
        side = self._side_stream(dy.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._gemm_tn(M, N, K, dy, ldd, x, ldx, dw)
        self._side_keep.append(dy)
        self._side_keep.append(x)

    def _conv(self, a: Act, fw, cout, R, S, stride, pad, stats_buf=None):
        B, H, W, C = a.shape
        Ho = (H + 2 * pad - R) // stride + 1
        Wo = (W + 2 * pad - S) // stride + 1
        y = self._empty(B, Ho, Wo, cout, device=a.t.device)
        d = self._desc(B, H, W, C, cout, R, S, stride, pad)
        bn = a.bn
        flops = 2.0 * B * Ho * Wo * cout * R * S * C
        es = y.element_size()
        nbytes = float(es * (B * H * W * C + cout * R * S * C + B * Ho * Wo * cout))  # algorithmic: x, w, y once
        if stats_buf is not None and bn is None:
            # BN statistics per segment (one launch for all G forward calls)
            det = DETERMINISTIC
            call("artsbir_conv2d_fwd_seg", d, ptr(a.t), ptr(fw), ptr(y), self._G, None if det else ptr(stats_buf),
                 _s(), kernel="auto", flops=flops, nbytes=nbytes,
                 tag=f"fwd {B}x{H}x{W}x{C}->{cout} {R}x{S}/{stride}")
            if det:  # fixed-order f64 sums of the stored output instead of epilogue atomics
                call("artsbir_bn_stats_det", self.dt, ptr(y), self._G, B // self._G * Ho * Wo, cout,
                     ptr(stats_buf), 2 * NSLOT * cout, _s())
            return y
        if bn is not None:
            raise NotImplementedError("BatchNorm is applied once by act_pool, not on the conv's load")
        call("artsbir_conv2d_fwd", d, ptr(a.t), ptr(fw), ptr(y), cout, 0, 0, None, None, None, 0,
             ptr(stats_buf), _s(), kernel="auto", flops=flops, nbytes=nbytes)
        return y

    def _bn(self, bnmod, stats_buf, count, train):
        """finalise the BN of every segment in order (running statistics are
        updated once per segment, as by the reference's consecutive calls)"""
        C = bnmod.num_features
        G = self._G
        if train:
            self._bn_gen += 1
        st = BNState(torch.empty(G, 4, C, dtype=torch.float32, device=bnmod.weight.device), float(count))
        call("artsbir_bn_finalize_seg", ptr(stats_buf) if train else None, G, 2 * NSLOT * C, C, float(count),
             ptr(bnmod.weight.detach()), ptr(bnmod.bias.detach()), ptr(bnmod.running_mean), ptr(bnmod.running_var),
             ptr(bnmod.num_batches_tracked) if train else None, BN_MOMENTUM, BN_EPS, 1 if train else 0,
             ptr(st.buf), _s())
        return st

    def _conv_bn(self, a, conv, bnmod, fw, stride, pad, train, stats):
        cout, _, R, S = conv.weight.shape
        sb = stats.take(cout * self._G) if train else None
        y = self._conv(a, fw, cout, R, S, stride, pad, sb)
        B, Ho, Wo, _ = y.shape
        return y, self._bn(bnmod, sb, (B // self._G) * Ho * Wo, train)

    def _act_pool(self, x, bn, relu, pool, colsum=False):
        """relu(bn(x)) (+ 2x2 avgpool), one launch for all G segments (segment s
        normalised with its own BN block).  colsum: also return the output's column
        sums per segment, [G][NSLOT][C] replica rows (the folded BN backward's
        1^T x of the conv that reads it)"""
        B, H, W, C = x.shape
        p = max(pool, 1)
        out = self._empty(B, H // p, W // p, C, device=x.device)
        G = bn.G if bn is not None else self._G
        cs = torch.zeros(G, NSLOT, C, dtype=torch.float32, device=x.device) if colsum else None
        call("artsbir_act_pool_colsum", self.dt, ptr(x), ptr(bn.block) if bn is not None else None, relu, pool, B, H,
             W, C, G, ptr(out), ptr(cs), _s(), kernel="act_pool_kernel",
             nbytes=float(x.element_size() * B * C * (H * W + (H // p) * (W // p))),
             tag=f"act_pool {B}x{H}x{W}x{C} pool{pool}")
        return (out, cs) if colsum else out

    # ------------------------------------------------ inference (folded BN)
    def bn_stats_changed(self):
        """the running statistics were written behind torch's back (e.g. a
        broadcast from another rank): the folded eval weights are stale"""
        self._bn_gen += 1

    def _eval_params_key(self):
        bns = [mod for mod in self.model.modules() if isinstance(mod, torch.nn.BatchNorm2d)]
        return (self._params_key(), self._bn_gen, tuple((b.running_mean.data_ptr(), b.running_mean._version,
                                           b.running_var._version, b.weight._version, b.bias._version) for b in bns))

    def _fold(self, conv, bn, ci_pad=None):
        """conv weight with the eval BatchNorm folded in, packed for the forward, and its bias"""
        w = conv.weight.detach().float().contiguous()
        co, ci, r, s = w.shape
        wf = torch.empty_like(w)
        bias = torch.empty(co, dtype=torch.float32, device=w.device)
        call("artsbir_bn_fold", ptr(w), co, ci * r * s, ptr(bn.weight.detach()), ptr(bn.bias.detach()),
             ptr(bn.running_mean), ptr(bn.running_var), float(bn.eps), ptr(wf), ptr(bias), _s())
        ci_pad = ci_pad or ci
        fw = self._empty(co, r, s, ci_pad, device=w.device)
        call("artsbir_pack_weight", self.dt, ptr(wf), co, ci, r, s, ci_pad, 0, 0, ptr(fw), _s())
        return fw, bias

    def _eval_packed(self):
        key = self._eval_params_key()
        if self._eval_key != key:
            m = self.model
            ev = {}
            blocks = []
            for blk in m.blocks():
                d = {"conv1": self._fold(blk.conv1, blk.bn1), "conv2": self._fold(blk.conv2, blk.bn2),
                     "conv3": self._fold(blk.conv3, blk.bn3)}
                if blk.downsample is not None:
                    d["down"] = self._fold(blk.downsample[1], blk.downsample[2])
                blocks.append(d)
            ev["blocks"] = blocks
            self._eval, self._eval_key = ev, key
        return self._eval

    def _conv_act(self, x, fb, conv, stride, pad, relu, res=None):
        fw, bias = fb
        cout, _, R, S = conv.weight.shape
        B, H, W, C = x.shape
        Ho = (H + 2 * pad - R) // stride + 1
        Wo = (W + 2 * pad - S) // stride + 1
        y = self._empty(B, Ho, Wo, cout, device=x.device)
        d = self._desc(B, H, W, C, cout, R, S, stride, pad)
        es = y.element_size()
        nbytes = float(es * (B * H * W * C + cout * R * S * C + B * Ho * Wo * cout * (2 if res is not None else 1)))
        call("artsbir_conv2d_fwd_act", d, ptr(x), ptr(fw), ptr(y), ptr(bias), ptr(res) if res is not None else None,
             1 if res is not None else 0, relu, _s(), kernel="auto", flops=2.0 * B * Ho * Wo * cout * R * S * C,
             nbytes=nbytes, tag=f"fwd_act {B}x{H}x{W}x{C}->{cout} {R}x{S}/{stride}")
        return y

    def _forward_eval(self, xs):
        """inference forward (models.py:344-360 with eval BatchNorm): conv + folded
        BN + ReLU (+ residual) per launch, AvgPool2d as a pooling pass"""
        m = self.model
        ev = self._eval_packed()
        pk = self.packed()
        G = len(xs)
        Bs, cin, R, R2 = xs[0].shape
        B = G * Bs
        dev = xs[0].device
        x0 = self._empty(B, R, R2, 8, device=dev)
        for i, xi in enumerate(xs):
            xi = xi.contiguous().float()
            call("artsbir_pack_input", self.dt, ptr(xi), Bs, cin, R, R2, _at(x0, i * Bs), _s())
        # the stem's few-channel convs stay on their direct kernels (sconv / hconv,
        # no bias epilogue) with the eval BN applied by act_pool: faster than the
        # GEMM kernel with a fused epilogue at 8 / 32 input channels
        self._G = 1
        (fw1, _), (fw2, _), (fw3, _) = pk["stem"]
        y1, b1 = self._conv_bn(Act(x0), m.conv1, m.bn1, fw1, 2, 1, False, None)
        y2, b2 = self._conv_bn(Act(self._act_pool(y1, b1, 1, 0)), m.conv2, m.bn2, fw2, 1, 1, False, None)
        y3, b3 = self._conv_bn(Act(self._act_pool(y2, b2, 1, 0)), m.conv3, m.bn3, fw3, 1, 1, False, None)
        h = self._act_pool(y3, b3, 1, 2)
        for blk, bp in zip(m.blocks(), ev["blocks"]):
            s = blk.stride
            a1 = self._conv_act(h, bp["conv1"], blk.conv1, 1, 0, 1)
            a2 = self._conv_act(a1, bp["conv2"], blk.conv2, 1, 1, 1)
            if s > 1:
                a2 = self._act_pool(a2, None, 0, s)
            if blk.downsample is not None:
                din = self._act_pool(h, None, 0, s) if s > 1 else h
                idn = self._conv_act(din, bp["down"], blk.downsample[1], 1, 0, 0)
            else:
                idn = h
            h = self._conv_act(a2, bp["conv3"], blk.conv3, 1, 0, 1, res=idn)
        out, _ = self._attnpool_fwd(m.attnpool, pk, h)
        return out

    # ---------------------------------------------------------------- forward
    def forward(self, x, train: bool, save: bool):
        """x: [B,3,R,R] or a list of G such batches (G separate reference forward
        calls run as one batch of G BN segments).  Returns ([G*B, out], ctx)."""
        xs = list(x) if isinstance(x, (list, tuple)) else [x]
        for xi in xs:
            if not xi.is_cuda:
                raise RuntimeError("ModifiedResNet on libartsbir_hip runs on the GPU: move model and input to cuda")
            if tuple(xi.shape) != tuple(xs[0].shape):
                raise ValueError("forward_branches: every branch needs the same input shape")
        G = len(xs)
        self._G = G
        _hip.lib().artsbir_set_deterministic(1 if DETERMINISTIC else 0)
        if not train and not save and FUSED_EVAL and type(self) is Engine:
            return self._forward_eval(xs), None
        m = self.model
        pk = self.packed()
        Bs, cin, R, R2 = xs[0].shape
        B = G * Bs
        dev = xs[0].device
        nstat = 2 * NSLOT * m.total_bn_channels() * G if train else 0
        stats = _Arena(torch.zeros(max(nstat, 1), dtype=torch.float32, device=dev), NSLOT * 2)
        ctx = {"train": train, "B": B, "G": G}

        # stem (models.py:345-350)
        x0 = self._empty(B, R, R2, 8, device=dev)
        for i, xi in enumerate(xs):
            xi = xi.contiguous().float()
            call("artsbir_pack_input", self.dt, ptr(xi), Bs, cin, R, R2, _at(x0, i * Bs), _s())
        (fw1, _), (fw2, _), (fw3, _) = pk["stem"]
        y1, b1 = self._conv_bn(Act(x0), m.conv1, m.bn1, fw1, 2, 1, train, stats)
        a1 = self._act_pool(y1, b1, 1, 0)
        y2, b2 = self._conv_bn(Act(a1), m.conv2, m.bn2, fw2, 1, 1, train, stats)
        a2 = self._act_pool(y2, b2, 1, 0)
        y3, b3 = self._conv_bn(Act(a2), m.conv3, m.bn3, fw3, 1, 1, train, stats)
        fold = train and save and self._fold_on()
        h_cs = None
        if fold:  # the stem output is the first block's downsample input: its column sums for the fold
            h, h_cs = self._act_pool(y3, b3, 1, 2, colsum=True)
        else:
            h = self._act_pool(y3, b3, 1, 2)
        if save:
            ctx["stem"] = dict(x0=x0, y1=y1, a1=a1, y2=y2, a2=a2, y3=y3, b1=b1, b2=b2, b3=b3)

        # residual stages (models.py:354-357)
        bctx = []
        blocks = m.blocks()
        for i, (blk, bp) in enumerate(zip(blocks, pk["blocks"])):
            # the next block's folded conv1 needs the column sums of its input
            h, c, h_cs = self._block_fwd(blk, bp, h, train, stats, fold=fold, h_cs=h_cs,
                                         out_cs=fold and self._fold1_on() and i + 1 < len(blocks))
            bctx.append(c if save else None)
        ctx["blocks"] = bctx

        # attention pool (models.py:249-272)
        out, actx = self._attnpool_fwd(m.attnpool, pk, h)
        if save:
            ctx["attn"] = actx
        return out, (ctx if save else None)

    def _fold_on(self):
        """whether the backward folds the block-output BN through conv3 / the
        downsample conv (it needs the column sums of their inputs from the
        forward).  Every block folds, in every mode: where the block-output BN
        reduction is not fused into the next block's data gradient (the
        encoder's last block; the deterministic mode, which reduces in a fixed
        order) a reduce-only pass supplies g and the reduction (_bn_reduce_g)"""
        return FOLD_BN[0] and type(self) is Engine

    def _fold1_on(self):
        """whether the backward folds bn1 through conv1 (the y-side fold; it needs
        the column sums of the block input from the forward, like _fold_on)"""
        return FOLD_BN1[0] and self._fold_on()

    def _block_fwd(self, blk, bp, h, train, stats, fold=False, h_cs=None, out_cs=False):
        B, H, W, Cin = h.shape
        s = blk.stride
        # BN+ReLU outputs are materialised once (bf16): cheaper than re-applying
        # them in every GEMM tile that reads them (9 taps x N-tiles for 3x3)
        y1, b1 = self._conv_bn(Act(h), blk.conv1, blk.bn1, bp["conv1"][0], 1, 0, train, stats)
        a1 = self._act_pool(y1, b1, 1, 0)
        y2, b2 = self._conv_bn(Act(a1), blk.conv2, blk.bn2, bp["conv2"][0], 1, 1, train, stats)
        cs2 = csd = None
        if fold:  # conv3's input with its column sums (the folded BN backward's 1^T x)
            p2, cs2 = self._act_pool(y2, b2, 1, s if s > 1 else 0, colsum=True)
        else:
            p2 = self._act_pool(y2, b2, 1, s if s > 1 else 0)
        c3in = Act(p2)
        y3, b3 = self._conv_bn(c3in, blk.conv3, blk.bn3, bp["conv3"][0], 1, 0, train, stats)
        yd = bd = pd = None
        if blk.downsample is not None:
            if s > 1:
                if fold:
                    pd, csd = self._act_pool(h, None, 0, s, colsum=True)
                else:
                    pd = self._act_pool(h, None, 0, s)
                din = pd
            else:
                din = h
                csd = h_cs
            yd, bd = self._conv_bn(Act(din), blk.downsample[1], blk.downsample[2], bp["down"][0], 1, 0, train, stats)
        out = torch.empty_like(y3)
        G = self._G
        Bs = B // G
        C = out.shape[-1]
        rows = out[0].numel() // C * Bs
        # bf16 training: the ReLU mask of the block output as bits for the fused
        # backward (kind 3), 1/16 of re-reading `out` there
        bits = None
        if train and _fuse_bnb() and MASK_BITS and self.dt == _hip.DT_BF16:
            bits = torch.empty(out.numel() // 8, dtype=torch.uint8, device=out.device)
        ocs = torch.zeros(G, NSLOT, C, dtype=torch.float32, device=out.device) if out_cs else None
        call("artsbir_block_out_colsum", self.dt, ptr(y3), ptr(b3.block), ptr(yd), ptr(bd.block) if bd else None,
             None if yd is not None else ptr(h), rows * G, C, G, ptr(out),
             bits.data_ptr() if bits is not None else None, ptr(ocs), _s(),
             kernel="block_out_kernel", nbytes=float(out.element_size() * rows * G * C * 3 + (rows * G * C // 8 if bits
                                                                                                  is not None else 0)),
             tag=f"block_out {rows * G}x{C}{' +colsum' if ocs is not None else ''}")
        ctx = dict(h=h, y1=y1, a1=a1, y2=y2, p2=p2, y3=y3, yd=yd, pd=pd, out=out, bits=bits, b1=b1, b2=b2, b3=b3,
                   bd=bd, cs2=cs2, csd=csd, h_cs=h_cs)
        return out, ctx, ocs

    def _attnpool_fwd(self, ap, pk, h):
        B, Hs, Ws, C = h.shape
        P = Hs * Ws
        Tk = P + 1
        dev = h.device
        heads = ap.num_heads
        D = ap.c_proj.weight.shape[0]
        tok = self._empty(B, Tk, C, device=dev)
        call("artsbir_tokens_fwd", self.dt, ptr(h), ptr(ap.positional_embedding.detach()), B, P, C, ptr(tok), _s())
        wkv, _, bkv = pk["kv"]
        kv = self._empty(B * Tk, 2 * C, device=dev)
        self._gemm_nt(B * Tk, 2 * C, C, tok, C, wkv, kv, 2 * C, 0, 0, bkv)
        wq, _, bq = pk["q"]
        q = torch.empty(B, C, dtype=torch.float32, device=dev)
        self._gemm_nt(B, C, C, tok, Tk * C, wq, q, C, 1, 0, bq)
        pm = torch.empty(B, heads, Tk, dtype=torch.float32, device=dev)
        o = self._empty(B, C, device=dev)
        call("artsbir_attnpool_fwd", self.dt, ptr(q), ptr(kv), B, C, heads, Tk, ptr(pm), ptr(o), _s())
        wc, _, bc = pk["c"]
        out = torch.empty(B, D, dtype=torch.float32, device=dev)
        self._gemm_nt(B, D, C, o, C, wc, out, D, 1, 0, bc)
        return out, dict(tok=tok, kv=kv, q=q, pm=pm, o=o, P=P, Tk=Tk, hw=(Hs, Ws))

    # --------------------------------------------------------------- backward
    def grad_buffer(self, device):
        gb = getattr(self, "_grads", None)
        if gb is None or gb.flat.device != device or gb.flat.numel() != sum(p.numel() for p in self.model.parameters()):
            gb = self._grads = GradBuffer(self.model, device)
        gb.attach()
        return gb

    def backward(self, ctx, dout: torch.Tensor):
        if ctx is None:
            raise RuntimeError("backward through a forward that did not save activations")
        if not ctx["train"]:
            raise NotImplementedError("backward is implemented for train-mode BatchNorm (as in train.py)")
        m = self.model
        pk = self.packed()
        self._G = G = ctx["G"]
        _hip.lib().artsbir_set_deterministic(1 if DETERMINISTIC else 0)
        dev = dout.device
        grads = self.grad_buffer(dev)
        ws = _Arena(torch.zeros(max(2 * NSLOT * m.total_bn_channels() * 2 * G, 1), dtype=torch.float32, device=dev),
                    NSLOT * 2)
        # the hook only sees a backward that carries every branch of the step
        # (one batched multi-branch pass); per-branch backwards accumulate and
        # are reduced after the last one by the hook's finish()
        hook = self.grad_hook if G > 1 else None
        streams = [torch.cuda.current_stream()] + ([self._side_stream(dev)] if OVERLAP_WGRAD else [])
        if hook is not None:
            hook.begin(grads.flat)
        dh = self._attnpool_bwd(m.attnpool, pk, ctx["attn"], dout.contiguous().float(), grads)
        blocks, bps, cs = m.blocks(), pk["blocks"], ctx["blocks"]
        if hook is not None:
            hook.ready(_param_ranges(grads, m.attnpool.parameters()), streams)
        fused = None
        for i in reversed(range(len(blocks))):
            prev = (blocks[i - 1], cs[i - 1]) if i > 0 else None
            dh, fused = self._block_bwd(blocks[i], bps[i], cs[i], dh, grads, ws, fused, prev)
            # block i+1 is final once block i is enqueued (block i's backward
            # still finishes the BN reduction handed over by block i+1)
            if hook is not None and i + 1 < len(blocks):
                hook.ready(_param_ranges(grads, blocks[i + 1].parameters()), streams)
        self._stem_bwd(m, pk, ctx["stem"], dh, grads, ws)
        if hook is not None:
            hook.end(streams)  # block 0, the stem and anything unreported
        if OVERLAP_WGRAD:
            torch.cuda.current_stream().wait_stream(self._side_stream(dev))
        self._side_keep = []
        return grads

    def _attnpool_bwd(self, ap, pk, c, dout, grads):
        tok, kv, q, pm, o = c["tok"], c["kv"], c["q"], c["pm"], c["o"]
        B, Tk, C = tok.shape
        P = c["P"]
        heads = ap.num_heads
        D = dout.shape[1]
        dev = dout.device
        call("artsbir_colsum", _hip.DT_F32, ptr(dout), B, D, D, ptr(grads[ap.c_proj.bias]), _s())
        if self.dtype == torch.float32:
            doutT = dout
        else:
            doutT = self._empty(B, D, device=dev)
            call("artsbir_cast", _hip.DT_F32, ptr(dout), self.dt, ptr(doutT), B * D, _s())
        # the head's weight gradients (c_proj, then q and k|v below) on the side
        # stream, idle at this point of the backward: the k|v one (B*Tk rows) is
        # ~0.65 ms that the main stream's data-gradient chain no longer waits for
        self._side_gemm_tn(B, D, C, doutT, D, o, C, grads[ap.c_proj.weight])
        _, wcT, _ = pk["c"]
        do = torch.empty(B, C, dtype=torch.float32, device=dev)
        self._gemm_nt(B, C, D, doutT, D, wcT, do, C, 1, 0, None)
        dq = self._empty(B, C, device=dev)
        dkv = self._empty(B * Tk, 2 * C, device=dev)
        call("artsbir_attnpool_bwd", self.dt, ptr(q), ptr(kv), ptr(pm), ptr(do), B, C, heads, Tk, ptr(dq), ptr(dkv),
             _s())
        call("artsbir_colsum", self.dt, ptr(dq), B, C, C, ptr(grads[ap.q_proj.bias]), _s())
        call("artsbir_colsum", self.dt, ptr(dkv), B * Tk, 2 * C, 2 * C, ptr(grads[ap.k_proj.bias]), _s())
        self._side_gemm_tn(B, C, C, dq, C, tok, Tk * C, grads[ap.q_proj.weight])
        self._side_gemm_tn(B * Tk, 2 * C, C, dkv, 2 * C, tok, C, grads[ap.k_proj.weight])
        _, wkvT, _ = pk["kv"]
        _, wqT, _ = pk["q"]
        Hs, Ws = c["hw"]
        dh = self._empty(B, Hs, Ws, C, device=dev)
        if self.dtype == torch.float32:
            dtok = torch.empty(B, Tk, C, dtype=torch.float32, device=dev)
            self._gemm_nt(B * Tk, C, 2 * C, dkv, 2 * C, wkvT, dtok, C, 1, 0, None)
            self._gemm_nt(B, C, C, dq, C, wqT, dtok, Tk * C, 1, 1, None)
            call("artsbir_colsum", _hip.DT_F32, ptr(dtok), B, Tk * C, Tk * C, ptr(grads[ap.positional_embedding]),
                 _s())
            call("artsbir_tokens_bwd", self.dt, ptr(dtok), B, P, C, ptr(dh), _s())
        else:
            # the token gradient of the key/value projections in the compute dtype
            # (the MFMA conv GEMM); the query projection's share of the mean token
            # (B rows) in f32 beside it, added where the two are consumed
            dtok = self._empty(B, Tk, C, device=dev)
            self._gemm_nt(B * Tk, C, 2 * C, dkv, 2 * C, wkvT, dtok, C, 0, 0, None)
            d0 = torch.empty(B, C, dtype=torch.float32, device=dev)
            self._gemm_nt(B, C, C, dq, C, wqT, d0, C, 1, 0, None)
            pos = grads[ap.positional_embedding]
            call("artsbir_colsum", self.dt, ptr(dtok), B, Tk * C, Tk * C, ptr(pos), _s())
            call("artsbir_colsum", _hip.DT_F32, ptr(d0), B, C, C, ptr(pos), _s())
            call("artsbir_tokens_bwd_ex", self.dt, ptr(dtok), ptr(d0), B, P, C, ptr(dh), _s())
        return dh

    def _seg_desc(self, kind, pool, targets, Bs, H, W, C):
        """a BN-backward descriptor covering all G segments in one launch
        (tensors advance by Bs images per segment, parameters by one block)"""
        desc = _hip.BnBwdDesc()
        desc.dtype = self.dt
        desc.kind = kind
        desc.pool = pool
        desc.ntarget = len(targets)
        for i, (y, st) in enumerate(targets):
            desc.y[i] = ptr(y)
            desc.mean[i] = ptr(st.mean)
            desc.istd[i] = ptr(st.istd)
        desc.B, desc.H, desc.W, desc.C = Bs, H, W, C
        desc.nseg = self._G
        desc.pstride, desc.cstride, desc.sstride = 4 * C, 3 * C, 2 * NSLOT * C
        return desc

    def _bn_bwd(self, kind, d, targets, bnmods, ws, grads, mask=None, mask_bn=None, pool=0, gout=None):
        """BatchNorm backward as a reduce pass + apply pass, each one launch over
        all G segments.  targets: list of (y, BNState); returns list of dy tensors"""
        y0 = targets[0][0]
        B, H, W, C = y0.shape
        G = self._G
        Bs = B // G
        dys = [torch.empty_like(y) for y, _ in targets]
        slots = [ws.take(C * G) for _ in targets]  # [G][NSLOT][2][C] per target
        desc = self._seg_desc(kind, pool, targets, Bs, H, W, C)
        desc.d = ptr(d)
        desc.mask = ptr(mask)
        desc.mask_bn = ptr(mask_bn.block) if mask_bn is not None else None
        for i in range(len(targets)):
            desc.slots[i] = ptr(slots[i])
        call("artsbir_bn_bwd_reduce", desc, _s(), kernel=f"bn_bwd_reduce_kernel<{kind}>",
             nbytes=float(y0.element_size() * B * H * W * C * (1.0 / max(pool, 1) ** 2 + len(targets)
                                                                 + (1 if kind == 0 else 0))),
             tag=f"bn_bwd_reduce k{kind} {B}x{H}x{W}x{C} t{len(targets)}")
        # one finalisation per target for all segments, then the apply
        coefs = self._bn_coefs(targets, bnmods, slots, grads, float(Bs * H * W))
        for i in range(len(targets)):
            desc.coef[i] = ptr(coefs[i])
            desc.dy[i] = ptr(dys[i])
        desc.gout = ptr(gout)
        call("artsbir_bn_bwd_apply", desc, _s(), kernel=f"bn_bwd_apply_kernel<{kind}>",
             nbytes=float(y0.element_size() * B * H * W * C * (1.0 / max(pool, 1) ** 2 + 2 * len(targets)
                                                                 + (1 if gout is not None else 0))),
             tag=f"bn_bwd_apply k{kind} {B}x{H}x{W}x{C} t{len(targets)}")
        return dys

    def _bn_reduce_g(self, d, targets, ws, mask=None, kind=0, mask_bn=None):
        """the reduce half of _bn_bwd: g = d * relu mask is written (kind 0: the
        block output's mask; kind 1: the BN before the ReLU, mask_bn) and Σg,
        Σg·x̂ of every target and segment go to the slots (fixed-order f64 in the
        deterministic mode), no apply pass — the BN backward is then folded
        through the 1x1 convs.  Returns (g, fused) in the form of a fused data
        gradient's hand-over (_bnb_fused_desc)."""
        y0 = targets[0][0]
        B, H, W, C = y0.shape
        G = self._G
        g = torch.empty_like(d)
        slots = [ws.take(C * G) for _ in targets]
        desc = self._seg_desc(kind, 0, targets, B // G, H, W, C)
        desc.d = ptr(d)
        desc.mask = ptr(mask)
        desc.mask_bn = ptr(mask_bn.block) if mask_bn is not None else None
        desc.gout = ptr(g)
        for i in range(len(targets)):
            desc.slots[i] = ptr(slots[i])
        call("artsbir_bn_bwd_reduce", desc, _s(), kernel=f"bn_bwd_reduce_kernel<{kind}>",
             nbytes=float(y0.element_size() * B * H * W * C * (2 + (kind == 0) + len(targets))),
             tag=f"bn_bwd_reduce k{kind} {B}x{H}x{W}x{C} t{len(targets)} +g")
        return g, (None, slots, targets)

    def _bn_coefs(self, targets, bnmods, slots, grads, count):
        """parameter gradients (+=) and apply coefficients [G][3][C] of every
        segment, one launch per BN target"""
        coefs = []
        for i, ((y, st), bnm) in enumerate(zip(targets, bnmods)):
            C = y.shape[-1]
            coef = torch.empty(self._G, 3, C, dtype=torch.float32, device=y.device)
            call("artsbir_bn_bwd_finalize_seg", ptr(slots[i]), self._G, 2 * NSLOT * C, C, count,
                 ptr(bnm.weight.detach()), ptr(st.buf[0, 1]), 4 * C, ptr(grads[bnm.weight]), ptr(grads[bnm.bias]),
                 ptr(coef), _s())
            coefs.append(coef)
        return coefs

    def _bnb_fused_desc(self, kind, targets, ws, mask=None, mask_bn=None):
        """descriptor of a BN-backward reduction fused into the data-gradient GEMM
        that produces its input gradient (all G segments; slots [G][NSLOT][2][C])"""
        y0 = targets[0][0]
        B, H, W, C = y0.shape
        desc = _hip.BnBwdDesc()
        desc.dtype = self.dt
        desc.kind = kind
        desc.pool = 0
        desc.mask = ptr(mask)
        desc.mask_bn = ptr(mask_bn.block) if mask_bn is not None else None
        desc.ntarget = len(targets)
        slots = []
        for i, (y, st) in enumerate(targets):
            desc.y[i] = ptr(y)
            desc.mean[i] = ptr(st.mean)
            desc.istd[i] = ptr(st.istd)
            sl = ws.take(C * self._G)
            slots.append(sl)
            desc.slots[i] = ptr(sl)
        desc.B, desc.H, desc.W, desc.C = B, H, W, C
        return desc, slots, targets

    def _bn_finish(self, g, fused, bnmods, grads):
        """apply pass of a fused BN-backward: g (masked) -> dy per target, one
        launch over all G segments"""
        _, slots, targets = fused
        y0 = targets[0][0]
        B, H, W, C = y0.shape
        G = self._G
        Bs = B // G
        dys = [torch.empty_like(y) for y, _ in targets]
        coefs = self._bn_coefs(targets, bnmods, slots, grads, float(Bs * H * W))
        desc = self._seg_desc(2, 0, targets, Bs, H, W, C)
        desc.d = ptr(g)
        for i in range(len(targets)):
            desc.coef[i] = ptr(coefs[i])
            desc.dy[i] = ptr(dys[i])
        call("artsbir_bn_bwd_apply", desc, _s(), kernel="bn_bwd_apply_kernel<2>",
             nbytes=float(y0.element_size() * B * H * W * C * (1 + 2 * len(targets))),
             tag=f"bn_bwd_apply k2 {B}x{H}x{W}x{C} t{len(targets)}")
        return dys

    def _side_stream(self, device):
        """the weight-gradient stream; with SIDE_CUS > 0 it may only use that many
        CUs (spread evenly over the chip), so the main stream's HBM-bound chain
        always finds free CUs while the MFMA-bound weight gradients run beside it"""
        st = getattr(self, "_side", None)
        want = (SIDE_CUS[0], SIDE_CONTIGUOUS[0])
        if st is None or st.device != device or getattr(self, "_side_cus", None) != want:
            if SIDE_CUS[0] > 0:
                st = self._side = cu_masked_stream(device, SIDE_CUS[0], contiguous=SIDE_CONTIGUOUS[0])
            else:
                st = self._side = torch.cuda.Stream(device=device)
            # the weight-gradient grids fill the side stream's CUs in whole rounds
            _hip.lib().artsbir_set_wgrad_cus(SIDE_CUS[0] if SIDE_CUS[0] > 0 else 256)
            self._side_cus = want
        return st

    def _wgrad(self, dy, a: Act, conv, stride, pad, grads, ci_pad=None):
        """weight gradient on a second stream: it only reads dy and the layer
        input and accumulates into its own slice of the gradient buffer, so it
        runs concurrently with the (HBM-bound) data-gradient / BatchNorm chain
        of the main stream; backward() joins the streams at the end."""
        if SKIP_WGRAD[0]:  # measurement only (tools/cu_mask_sweep.py): the main stream's critical path
            return
        if not OVERLAP_WGRAD or (WGRAD_MAIN and WGRAD_MAIN == ("1x1" if conv.weight.shape[2] == 1 else "3x3")):
            return self._wgrad_sync(dy, a, conv, stride, pad, grads, ci_pad)
        main = torch.cuda.current_stream()
        side = self._side_stream(dy.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self._wgrad_sync(dy, a, conv, stride, pad, grads, ci_pad)
        # the caching allocator must not hand these to the main stream before
        # the side stream is done with them: they stay referenced until the
        # backward's final join (main waits for side), after which their blocks
        # return to the main stream's pool in stream order.  (record_stream
        # would instead tie every block to the side stream's progress, so the
        # allocator keeps mallocing fresh blocks — ~60 hipMallocs a step, the
        # pool creeping towards the 288 GB capacity, and an occasional
        # seconds-long stall when the driver has to make room.)
        self._side_keep.append(dy)
        self._side_keep.append(a.t)

    def _wgrad_sync(self, dy, a: Act, conv, stride, pad, grads, ci_pad=None):
        B, H, W, C = a.shape
        co, ci, R, S = conv.weight.shape
        d = self._desc(B, H, W, C, co, R, S, stride, pad)
        bn = a.bn
        g = grads[conv.weight]
        if R == 1 and S == 1 and C == ci:
            target = g
        else:
            target = torch.zeros(co, R, S, C, dtype=torch.float32, device=dy.device)
        Ho, Wo = dy.shape[1], dy.shape[2]
        if bn is not None:
            raise NotImplementedError("BatchNorm is applied once by act_pool, not on the wgrad's load")
        call("artsbir_conv2d_wgrad", d, ptr(dy), ptr(a.t), None, None, 0, ptr(target), _s(), kernel="auto",
             flops=2.0 * B * Ho * Wo * co * R * S * C, tag=f"wgrad {B}x{H}x{W}x{C}->{co} {R}x{S}/{stride}",
             nbytes=float(dy.element_size() * (B * Ho * Wo * co + B * H * W * C) + 4 * co * R * S * C))
        if target is not g:
            call("artsbir_unpack_wgrad", ptr(target), co, ci, R, S, C, ptr(g), _s())

    def _wgrad_pre(self, dy, a, conv, stride, pad, grads):
        """issue a layer's weight gradient now, or hold it (WGRAD_DEFER) until
        _wgrad_post is called after the layer's data gradient"""
        k = WGRAD_DEFER[0]
        if k and (k == "all" or k == ("1x1" if conv.weight.shape[2] == 1 else "3x3")):
            return (dy, a, conv, stride, pad, grads)
        self._wgrad(dy, a, conv, stride, pad, grads)
        return None

    def _wgrad_post(self, held):
        if held is not None:
            self._wgrad(*held)

    def _dgrad(self, dy, dw, conv, pad, out_shape, res=None, res_mode=0, fused=None):
        B, H, W, C = out_shape
        co, _, R, S = conv.weight.shape
        dx = self._empty(B, H, W, C, device=dy.device)
        d = self._desc(B, H, W, C, co, R, S, 1, pad)
        flops = 2.0 * B * H * W * C * R * S * co
        es = dx.element_size()
        px = B * H * W
        # algorithmic bytes: dy, w, dx once; residual; BN-backward operands (y_t, mask)
        nb = px * co + co * R * S * C + px * C + (px * C if res_mode == 1 else px * C // 4 if res_mode == 2 else 0)
        if fused is not None:
            nb += px * C * (fused[0].ntarget + {0: 1.0, 3: 1.0 / 16}.get(fused[0].kind, 0.0))
        nbytes = float(es * nb)
        if fused is None:
            call("artsbir_conv2d_dgrad", d, ptr(dy), ptr(dw), ptr(dx), ptr(res), res_mode, _s(),
                 kernel="auto", flops=flops, nbytes=nbytes, tag=f"dgrad {B}x{H}x{W}x{co}->{C} {R}x{S} res{res_mode}")
        else:
            call("artsbir_conv2d_dgrad_bnb", d, ptr(dy), ptr(dw), ptr(dx), ptr(res), res_mode,
                 ctypes.byref(fused[0]), self._G, 4 * C, _s(), kernel="auto", flops=flops, nbytes=nbytes,
                 tag=f"dgrad+bn{fused[0].kind} {B}x{H}x{W}x{co}->{C} {R}x{S} res{res_mode}")
        return dx

    # ------------------------------------ BatchNorm backward folded through a 1x1 conv
    def _fold_weights(self, packs, conv, coef, st: BNState):
        """per-segment weights [G][Ci][Co + Ci] and bias [G][Ci] of the folded data
        gradient (artsbir_bn_fold_bwd_prep): the g side diag(c1) W, the x side
        W^T diag(b') W, the bias k W"""
        _, wd = packs
        co, ci = conv.weight.shape[:2]
        G = self._G
        dev = wd.device
        wout = self._empty(G, ci, co + ci, device=dev)
        bias = torch.empty(G, ci, dtype=torch.float32, device=dev)
        amat = self._empty(G, ci, co, device=dev)
        es = wout.element_size()
        call("artsbir_bn_fold_bwd_prep", self.dt, co, ci, ptr(wd), ptr(coef), ptr(st.buf), 4 * co, G, ptr(wout),
             ptr(bias), ptr(amat), _s(), kernel="fold_prep+gemm", flops=2.0 * G * ci * ci * co,
             nbytes=float(es * (ci * co * (1 + 2 * G) + G * ci * (co + ci))), tag=f"fold_prep {co}->{ci} x{G}")
        return wout, bias

    def _dgrad_fold(self, g, x, fold, conv, fused=None):
        """dx = [g | x] w_s^T + bias_s (artsbir_conv1x1_dgrad_fold): the data
        gradient of a 1x1 conv through the BatchNorm after it, from the masked
        gradient g at the BN output and the conv input x"""
        wout, bias = fold
        B, H, W, ci = x.shape
        co = conv.weight.shape[0]
        dx = self._empty(B, H, W, ci, device=x.device)
        d = self._desc(B, H, W, ci, co, 1, 1, 1, 0)
        px = B * H * W
        es = dx.element_size()
        nb = px * co + px * ci + self._G * ci * (co + ci) + px * ci + (px * ci if fused is not None else 0)
        call("artsbir_conv1x1_dgrad_fold", d, ptr(g), ptr(x), ptr(wout), ptr(bias), ptr(dx),
             ctypes.byref(fused[0]) if fused is not None else None, self._G, 4 * ci, _s(), kernel="auto",
             flops=2.0 * px * ci * (co + ci), nbytes=float(es * nb),
             tag=f"dgrad_fold{'+bn1' if fused is not None else ''} {B}x{H}x{W}x{co}+{ci}->{ci}")
        return dx

    def _fold_wg_ok(self, x, conv):
        """whether the fold's data gradient also produces its weight-gradient
        operands in the same pass (artsbir_conv1x1_dgrad_fold_wg's one-kernel
        shapes: layer 1, Ci 64 under Co 256, whole 256-pixel tiles per segment)"""
        B, H, W, ci = x.shape
        return (FOLD_WG[0] and not SKIP_WGRAD[0] and self.dtype == torch.bfloat16 and ci == 64
                and conv.weight.shape[0] == 256 and (B // self._G) * H * W % 256 == 0)

    def _dgrad_fold_wg(self, g, x, fold, conv, fw, coef, st: BNState, grads, cs=None, fused=None):
        """_dgrad_fold whose kernel also accumulates g^T x and x^T x per segment
        (artsbir_conv1x1_dgrad_fold_wg): the weight gradient then needs only the
        small combine on the side stream, g and x are read once"""
        wout, bias = fold
        B, H, W, ci = x.shape
        co = conv.weight.shape[0]
        G = self._G
        dx = self._empty(B, H, W, ci, device=x.device)
        buf = torch.zeros(G * (co + ci) * ci, dtype=torch.float32, device=x.device)
        P, gram = buf[:G * co * ci].view(G, co, ci), buf[G * co * ci:].view(G, ci, ci)
        d = self._desc(B, H, W, ci, co, 1, 1, 1, 0)
        px = B * H * W
        es = dx.element_size()
        nb = es * (px * co + px * ci + G * ci * (co + ci) + px * ci + (px * ci if fused is not None else 0)) \
            + 4 * G * (co + ci) * ci
        call("artsbir_conv1x1_dgrad_fold_wg", d, ptr(g), ptr(x), ptr(wout), ptr(bias), ptr(dx),
             ctypes.byref(fused[0]) if fused is not None else None, G, 4 * ci, ptr(P), ptr(gram), _s(),
             kernel="auto", flops=4.0 * px * ci * (co + ci), nbytes=float(nb),
             tag=f"dgrad_fold_wg{'+bn1' if fused is not None else ''} {B}x{H}x{W}x{co}+{ci}->{ci}")
        self._wgrad_fold(g, x, conv, fw, coef, st, grads, cs, pg=(P, gram, buf))
        return dx

    def _wgrad_fold(self, g, x, conv, fw, coef, st: BNState, grads, cs=None, pg=None):
        """weight gradient of a 1x1 conv through the BatchNorm after it (side
        stream): per segment g^T x, the Gram matrix x^T x and the column sums of
        x (cs [G][slots][Ci], from the forward's act_pool, else a column-sum pass
        here), combined by artsbir_bn_fold_wgrad_combine into the gradient buffer.
        pg: (P, Gram, buffer) already accumulated on the main stream by
        _dgrad_fold_wg (only the combine runs here)"""
        if SKIP_WGRAD[0]:
            return
        main = torch.cuda.current_stream()
        side = self._side_stream(g.device) if OVERLAP_WGRAD else main
        if side is not main:
            side.wait_stream(main)
        G = self._G
        B, H, W, ci = x.shape
        co = conv.weight.shape[0]
        Bs = B // G
        Ms = Bs * H * W
        es = x.element_size()
        with torch.cuda.stream(side):
            # [P | Gram | colsums] of every segment in one zeroed buffer, then the
            # combine's workspace (W in f32, T = W Gram)
            nP, nG = G * co * ci, G * ci * ci
            own_cs = cs is None
            if pg is not None:
                P, gram, buf = pg
                if own_cs:
                    cs = torch.zeros(G, 1, ci, dtype=torch.float32, device=x.device)
                    self._side_keep.append(cs)
            else:
                buf = torch.zeros(nP + nG + (G * ci if own_cs else 0), dtype=torch.float32, device=x.device)
                P, gram = buf[:nP].view(G, co, ci), buf[nP:nP + nG].view(G, ci, ci)
                if own_cs:
                    cs = buf[nP + nG:].view(G, 1, ci)
            wsp = torch.empty(co * ci * (G + 1), dtype=torch.float32, device=x.device)
            for s in range(G):
                gs, xs = g[s * Bs:(s + 1) * Bs], x[s * Bs:(s + 1) * Bs]
                # g_s^T x_s and x_s^T x_s, one launch (the x rows read once for both)
                if pg is None:
                    call("artsbir_gemm_tn2", self.dt, Ms, co, ci, ci, ptr(gs), co, ptr(xs), ci, ptr(xs), ci,
                         ptr(P[s]), ptr(gram[s]), _s(), kernel="auto", flops=2.0 * Ms * (co + ci) * ci,
                         nbytes=float(es * Ms * (co + ci) + 4 * (co + ci) * ci), tag=f"wgrad_fold {Ms}x{co}+{ci}x{ci}")
                if own_cs:
                    call("artsbir_colsum", self.dt, ptr(xs), Ms, ci, ci, ptr(cs[s]), _s(), kernel="colsum_kernel",
                         nbytes=float(es * Ms * ci), tag=f"colsum {Ms}x{ci}")
            call("artsbir_bn_fold_wgrad_combine", self.dt, co, ci, G, ptr(P), ptr(gram), ptr(cs), cs.shape[1], ptr(fw),
                 ptr(coef), ptr(st.buf), 4 * co, ptr(grads[conv.weight]), ptr(wsp), _s(), kernel="fold_combine",
                 flops=2.0 * G * co * ci * ci, nbytes=float(4 * (G * (co * ci + ci * ci) + 3 * co * ci)),
                 tag=f"fold_combine {co}x{ci}")
        if side is not main:
            self._side_keep.extend([g, x, coef, st.buf, buf, wsp, cs])

    # ------------------------- bn1 folded through conv1 with its own input (y-side)
    def _fold_weights_y(self, packs, conv, coef, st: BNState):
        """per-segment weights [G][Ci][2 Co] and bias [G][Ci] of the y-side fold
        (artsbir_bn_fold_bwd_prep_y): the g side diag(c1) W, the y side
        diag(b') W, the bias k W"""
        _, wd = packs
        co, ci = conv.weight.shape[:2]
        G = self._G
        wout = self._empty(G, ci, 2 * co, device=wd.device)
        bias = torch.empty(G, ci, dtype=torch.float32, device=wd.device)
        es = wout.element_size()
        call("artsbir_bn_fold_bwd_prep_y", self.dt, co, ci, ptr(wd), ptr(coef), ptr(st.buf), 4 * co, G, ptr(wout),
             ptr(bias), _s(), kernel="fold_prep_y_kernel", nbytes=float(es * ci * co * (1 + 2 * G) + 4 * G * ci),
             tag=f"fold_prep_y {co}->{ci} x{G}")
        return wout, bias

    def _dgrad_fold_y(self, g, y, fold, conv, out_shape, res, res_mode, fused=None):
        """dx = [g | y] w_s^T + bias_s (+ residual) (artsbir_conv1x1_dgrad_fold_y):
        the data gradient of a 1x1 conv through the BatchNorm after it, from the
        masked gradient g at the BN output and the BN input y (the conv output)"""
        wout, bias = fold
        B, H, W, ci = out_shape
        co = conv.weight.shape[0]
        dx = self._empty(B, H, W, ci, device=g.device)
        d = self._desc(B, H, W, ci, co, 1, 1, 1, 0)
        px = B * H * W
        es = dx.element_size()
        nb = 2 * px * co + self._G * ci * 2 * co + px * ci + (px * ci if res_mode == 1 else
                                                                px * ci // 4 if res_mode == 2 else 0)
        if fused is not None:
            nb += px * ci * (fused[0].ntarget + {0: 1.0, 3: 1.0 / 16}.get(fused[0].kind, 0.0))
        call("artsbir_conv1x1_dgrad_fold_y", d, ptr(g), ptr(y), ptr(wout), ptr(bias), ptr(dx), ptr(res), res_mode,
             ctypes.byref(fused[0]) if fused is not None else None, self._G, 4 * ci, _s(), kernel="auto",
             flops=2.0 * px * ci * 2 * co, nbytes=float(es * nb),
             tag=f"dgrad_fold_y{'+bn' + str(fused[0].kind) if fused is not None else ''} {B}x{H}x{W}x{co}+{co}->{ci} "
                 f"res{res_mode}")
        return dx

    def _wgrad_fold_y(self, g, y, x, conv, coef, st: BNState, grads, cs=None):
        """weight gradient of a 1x1 conv through the BatchNorm after it, y-side
        (side stream): per segment g^T x and y^T x in one launch
        (artsbir_gemm_tn2), combined with the column sums of x (cs [G][slots][Ci]
        from the forward's block_out, else a column-sum pass here) by
        artsbir_bn_fold_wgrad_combine_y into the gradient buffer"""
        if SKIP_WGRAD[0]:
            return
        main = torch.cuda.current_stream()
        side = self._side_stream(g.device) if OVERLAP_WGRAD else main
        if side is not main:
            side.wait_stream(main)
        G = self._G
        B, H, W, ci = x.shape
        co = conv.weight.shape[0]
        Bs = B // G
        Ms = Bs * H * W
        es = x.element_size()
        with torch.cuda.stream(side):
            own_cs = cs is None
            buf = torch.zeros(2 * G * co * ci + (G * ci if own_cs else 0), dtype=torch.float32, device=x.device)
            P, Q = buf[:G * co * ci].view(G, co, ci), buf[G * co * ci:2 * G * co * ci].view(G, co, ci)
            if own_cs:
                cs = buf[2 * G * co * ci:].view(G, 1, ci)
            for s in range(G):
                gs, ys, xs = g[s * Bs:(s + 1) * Bs], y[s * Bs:(s + 1) * Bs], x[s * Bs:(s + 1) * Bs]
                call("artsbir_gemm_tn2", self.dt, Ms, co, co, ci, ptr(gs), co, ptr(ys), co, ptr(xs), ci,
                     ptr(P[s]), ptr(Q[s]), _s(), kernel="auto", flops=4.0 * Ms * co * ci,
                     nbytes=float(es * Ms * (2 * co + ci) + 8 * co * ci), tag=f"wgrad_fold_y {Ms}x{co}+{co}x{ci}")
                if own_cs:
                    call("artsbir_colsum", self.dt, ptr(xs), Ms, ci, ci, ptr(cs[s]), _s(), kernel="colsum_kernel",
                         nbytes=float(es * Ms * ci), tag=f"colsum {Ms}x{ci}")
            call("artsbir_bn_fold_wgrad_combine_y", co, ci, G, ptr(P), ptr(Q), ptr(cs), cs.shape[1], ptr(coef),
                 ptr(st.buf), 4 * co, ptr(grads[conv.weight]), _s(), kernel="fold_wgrad_combine_kernel",
                 nbytes=float(4 * (2 * G * co * ci + 2 * co * ci)), tag=f"fold_combine_y {co}x{ci}")
        if side is not main:
            self._side_keep.extend([g, y, x, coef, st.buf, buf, cs])

    def _block_bwd(self, blk, bp, c, dout, grads, ws, fused_res=None, prev=None):
        """backward of one Bottleneck.  dout: gradient of the block output, or —
        when fused_res is given — g = dout * relu-mask with the block-output BN
        reduction already done by the producing data-gradient GEMM.  prev: the
        (Bottleneck, ctx) feeding this block, whose output BN reduction is fused
        into this block's last data gradient.  Returns (dh, fused for prev)."""
        h, y1, y2, p2, y3, yd, pd, out = (c[k] for k in ("h", "y1", "y2", "p2", "y3", "yd", "pd", "out"))
        b1, b2, b3, bd = c["b1"], c["b2"], c["b3"], c["bd"]
        s = blk.stride
        has_ds = blk.downsample is not None
        bnmods = [blk.bn3] + ([blk.downsample[2]] if has_ds else [])
        # the block-output BN backward folded through conv3 / the downsample conv
        # (csrc/fold.hip): no dy3 / dyd tensors, their apply pass and re-reads gone
        fold = fused_res is not None and FOLD_BN[0]
        dys = coefs = None
        if fused_res is None and self._fold_on():
            # no data gradient reduced this BN for us (the last block; the
            # deterministic mode): a reduce-only pass, then the same fold
            targets = [(y3, b3)] + ([(yd, bd)] if has_ds else [])
            dout, fused_res = self._bn_reduce_g(dout, targets, ws, out)
            fold = True
        if fold:
            _, slots, targets = fused_res
            B3, H3, W3, _ = y3.shape
            coefs = self._bn_coefs(targets, bnmods, slots, grads, float(B3 // self._G * H3 * W3))
            gid = dout
        elif fused_res is not None:
            dys = self._bn_finish(dout, fused_res, bnmods, grads)
            gid = dout  # the identity branch's gradient is g itself
        else:
            targets = [(y3, b3)] + ([(yd, bd)] if has_ds else [])
            gid = None if has_ds else torch.empty_like(dout)
            dys = self._bn_bwd(0, dout, targets, bnmods, ws, grads, mask=out, gout=gid)
        c3in = Act(p2)
        c3out = c3in.shape[:3] + (blk.conv3.weight.shape[1],)
        if fold:
            fw3 = self._fold_weights(bp["conv3"], blk.conv3, coefs[0], b3)
            wg3 = self._fold_wg_ok(p2, blk.conv3)
            wargs = (blk.conv3, bp["conv3"][0], coefs[0], b3, grads, c.get("cs2"))
            if not wg3:
                self._wgrad_fold(dout, p2, *wargs)
            f2 = self._bnb_fused_desc(1, [(y2, b2)], ws, mask_bn=b2) if s == 1 and _fuse_bnb() else None
            if wg3:
                g2 = self._dgrad_fold_wg(dout, p2, fw3, *wargs, fused=f2)
            else:
                g2 = self._dgrad_fold(dout, p2, fw3, blk.conv3, fused=f2)
            if f2 is not None:
                dy2, = self._bn_finish(g2, f2, [blk.bn2], grads)
            else:
                dy2, = self._bn_bwd(1, g2, [(y2, b2)], [blk.bn2], ws, grads, mask_bn=b2, pool=s if s > 1 else 0)
        else:
            dy3 = dys[0]
            held = self._wgrad_pre(dy3, c3in, blk.conv3, 1, 0, grads)
            if s == 1 and _fuse_bnb():
                f2 = self._bnb_fused_desc(1, [(y2, b2)], ws, mask_bn=b2)
                g2 = self._dgrad(dy3, bp["conv3"][1], blk.conv3, 0, c3out, fused=f2)
                self._wgrad_post(held)
                dy2, = self._bn_finish(g2, f2, [blk.bn2], grads)
            else:
                dp = self._dgrad(dy3, bp["conv3"][1], blk.conv3, 0, c3out)
                self._wgrad_post(held)
                dy2, = self._bn_bwd(1, dp, [(y2, b2)], [blk.bn2], ws, grads, mask_bn=b2, pool=s if s > 1 else 0)
        held = self._wgrad_pre(dy2, Act(c["a1"]), blk.conv2, 1, 1, grads)
        # bn1 folded through conv1 with its input y1 (models.py:198-199): no dy1
        fold1 = fold and self._fold1_on()
        held1 = None
        if fold1:
            if _fuse_bnb():
                f1 = self._bnb_fused_desc(1, [(y1, b1)], ws, mask_bn=b1)
                g1 = self._dgrad(dy2, bp["conv2"][1], blk.conv2, 1, y1.shape, fused=f1)
            else:  # deterministic: the fixed-order reduce-only pass writes g1
                da1 = self._dgrad(dy2, bp["conv2"][1], blk.conv2, 1, y1.shape)
                g1, f1 = self._bn_reduce_g(da1, [(y1, b1)], ws, kind=1, mask_bn=b1)
            self._wgrad_post(held)
            B1, H1, W1, _ = y1.shape
            coef1, = self._bn_coefs([(y1, b1)], [blk.bn1], f1[1], grads, float(B1 // self._G * H1 * W1))
            fw1 = self._fold_weights_y(bp["conv1"], blk.conv1, coef1, b1)
            self._wgrad_fold_y(g1, y1, h, blk.conv1, coef1, b1, grads, c.get("h_cs"))
        elif _fuse_bnb():
            f1 = self._bnb_fused_desc(1, [(y1, b1)], ws, mask_bn=b1)
            g1 = self._dgrad(dy2, bp["conv2"][1], blk.conv2, 1, y1.shape, fused=f1)
            self._wgrad_post(held)
            dy1, = self._bn_finish(g1, f1, [blk.bn1], grads)
        else:
            da1 = self._dgrad(dy2, bp["conv2"][1], blk.conv2, 1, y1.shape)
            self._wgrad_post(held)
            dy1, = self._bn_bwd(1, da1, [(y1, b1)], [blk.bn1], ws, grads, mask_bn=b1)
        if not fold1:
            held1 = self._wgrad_pre(dy1, Act(h), blk.conv1, 1, 0, grads)
        if has_ds:
            din = pd if s > 1 else h
            dconv = blk.downsample[1]
            if fold:
                fwd_ = self._fold_weights(bp["down"], dconv, coefs[1], bd)
                wargs = (dconv, bp["down"][0], coefs[1], bd, grads, c.get("csd"))
                if self._fold_wg_ok(din, dconv):
                    res = self._dgrad_fold_wg(dout, din, fwd_, *wargs)
                else:
                    self._wgrad_fold(dout, din, *wargs)
                    res = self._dgrad_fold(dout, din, fwd_, dconv)
            else:
                dyd = dys[1]
                held = self._wgrad_pre(dyd, Act(din), dconv, 1, 0, grads)
                res = self._dgrad(dyd, bp["down"][1], dconv, 0, din.shape)
                self._wgrad_post(held)
            res_mode = 2 if s > 1 else 1
        else:
            res, res_mode = gid, 1
        fprev = None
        if prev is not None and _fuse_bnb():
            pblk, pc = prev
            ptargets = [(pc["y3"], pc["b3"])] + ([(pc["yd"], pc["bd"])] if pblk.downsample is not None else [])
            if pc.get("bits") is not None:
                fprev = self._bnb_fused_desc(3, ptargets, ws, mask=pc["bits"])
            else:
                fprev = self._bnb_fused_desc(0, ptargets, ws, mask=pc["out"])
        if fold1:
            dh = self._dgrad_fold_y(g1, y1, fw1, blk.conv1, h.shape, res, res_mode, fused=fprev)
        else:
            dh = self._dgrad(dy1, bp["conv1"][1], blk.conv1, 0, h.shape, res=res, res_mode=res_mode, fused=fprev)
            self._wgrad_post(held1)
        return dh, fprev

    def _stem_bwd(self, m, pk, c, dh, grads, ws):
        x0, y1, y2, y3, b1, b2, b3 = (c[k] for k in ("x0", "y1", "y2", "y3", "b1", "b2", "b3"))
        (_, _), (_, dw2), (_, dw3) = pk["stem"]
        dy3, = self._bn_bwd(1, dh, [(y3, b3)], [m.bn3], ws, grads, mask_bn=b3, pool=2)
        held = self._wgrad_pre(dy3, Act(c["a2"]), m.conv3, 1, 1, grads)
        if _fuse_bnb():
            f2 = self._bnb_fused_desc(1, [(y2, b2)], ws, mask_bn=b2)
            g2 = self._dgrad(dy3, dw3, m.conv3, 1, y2.shape, fused=f2)
            self._wgrad_post(held)
            dy2, = self._bn_finish(g2, f2, [m.bn2], grads)
        else:
            da2 = self._dgrad(dy3, dw3, m.conv3, 1, y2.shape)
            self._wgrad_post(held)
            dy2, = self._bn_bwd(1, da2, [(y2, b2)], [m.bn2], ws, grads, mask_bn=b2)
        held = self._wgrad_pre(dy2, Act(c["a1"]), m.conv2, 1, 1, grads)
        if _fuse_bnb():
            f1 = self._bnb_fused_desc(1, [(y1, b1)], ws, mask_bn=b1)
            g1 = self._dgrad(dy2, dw2, m.conv2, 1, y1.shape, fused=f1)
            self._wgrad_post(held)
            dy1, = self._bn_finish(g1, f1, [m.bn1], grads)
        else:
            da1 = self._dgrad(dy2, dw2, m.conv2, 1, y1.shape)
            self._wgrad_post(held)
            dy1, = self._bn_bwd(1, da1, [(y1, b1)], [m.bn1], ws, grads, mask_bn=b1)
        # the stem conv (models.py:310) has no data gradient, so the main stream
        # has nothing left to do: its weight gradient runs there, beside the side
        # stream's last ones, instead of queued behind them while main idles
        # (0.6 ms at the end of the C2 step, profiles/r6_trace_gaps.txt)
        if not STEM_WGRAD_MAIN:
            self._wgrad(dy1, Act(x0), m.conv1, 2, 1, grads)
        elif not SKIP_WGRAD[0]:
            self._wgrad_sync(dy1, Act(x0), m.conv1, 2, 1, grads)


class _Arena:
    """Bump allocator of per-channel slot blocks out of one zeroed f32 buffer."""

    def __init__(self, buf, per_channel):
        self.buf, self.per, self.off = buf, per_channel, 0

    def take(self, C):
        n = self.per * C
        v = self.buf[self.off:self.off + n]
        self.off += n
        if self.off > self.buf.numel():
            raise RuntimeError("statistics arena overflow")
        return v


def _module_grad_order(mod):
    """gradient-buffer order of a standalone submodule: an attention pool keeps
    k/v weights and biases adjacent (its fused K|V GEMMs write both at once)"""
    kv = []
    if hasattr(mod, "k_proj") and hasattr(mod, "v_proj"):
        kv = [mod.k_proj.weight, mod.v_proj.weight, mod.k_proj.bias, mod.v_proj.bias]
    ids = {id(p) for p in kv}
    return kv + [p for p in mod.parameters() if id(p) not in ids]


class ModuleEngine(Engine):
    """A Bottleneck or AttentionPool2d called on its own — the reference's
    submodule forwards (models.py:223-236, 249-272), e.g. a block probed in
    isolation — runs on the same kernels as the encoder: NCHW f32 in and out
    (NHWC compute layout inside), one autograd node per call, parameter
    gradients accumulated into param.grad (views of a per-module buffer)."""

    def _pack_all(self):
        m = self.model
        if hasattr(m, "conv3"):  # Bottleneck
            d = {"conv1": self._pack_conv(m.conv1), "conv2": self._pack_conv(m.conv2),
                 "conv3": self._pack_conv(m.conv3)}
            if m.downsample is not None:
                d["down"] = self._pack_conv(m.downsample[1])
            return d
        dev = m.k_proj.weight.device
        return {"kv": self._pack_linear_pair([m.k_proj, m.v_proj], dev), "q": self._pack_linear_pair([m.q_proj], dev),
                "c": self._pack_linear_pair([m.c_proj], dev)}

    def module_forward(self, x, train: bool):
        if not x.is_cuda:
            raise RuntimeError("libartsbir_hip modules run on the GPU: move module and input to cuda")
        if x.dim() != 4:
            raise ValueError(f"expected NCHW input, got shape {tuple(x.shape)}")
        self._G = 1
        _hip.lib().artsbir_set_deterministic(1 if DETERMINISTIC else 0)
        m = self.model
        pk = self.packed()
        h = x.detach().permute(0, 2, 3, 1).contiguous().to(self.dtype)
        if hasattr(m, "conv3"):
            nbn = sum(b.num_features for b in m.modules() if isinstance(b, torch.nn.BatchNorm2d))
            stats = _Arena(torch.zeros(max(2 * NSLOT * nbn, 1), dtype=torch.float32, device=x.device), NSLOT * 2)
            out, c, _ = self._block_fwd(m, pk, h, train, stats)
            return out.permute(0, 3, 1, 2).float().contiguous(), {"train": train, "c": c}
        out, c = self._attnpool_fwd(m, pk, h)
        return out.float(), {"train": train, "c": c}

    def module_backward(self, state, dout):
        if not state["train"]:
            raise NotImplementedError("backward is implemented for train-mode BatchNorm (as in train.py)")
        m = self.model
        pk = self.packed()
        self._G = 1
        dev = dout.device
        grads = self.grad_buffer(dev)
        if hasattr(m, "conv3"):
            nbn = sum(b.num_features for b in m.modules() if isinstance(b, torch.nn.BatchNorm2d))
            ws = _Arena(torch.zeros(max(2 * NSLOT * nbn * 2, 1), dtype=torch.float32, device=dev), NSLOT * 2)
            d = dout.permute(0, 2, 3, 1).contiguous().to(self.dtype)
            dh, _ = self._block_bwd(m, pk, state["c"], d, grads, ws, None, None)
        else:
            dh = self._attnpool_bwd(m, pk, state["c"], dout.contiguous().float(), grads)
        if OVERLAP_WGRAD:
            torch.cuda.current_stream().wait_stream(self._side_stream(dev))
        self._side_keep = []
        return dh.permute(0, 3, 1, 2).float().contiguous()


def _param_ranges(grads, params):
    """[lo, hi) element ranges of the gradient buffer holding params' gradients"""
    base = grads.flat.data_ptr()
    es = grads.flat.element_size()
    out = []
    for p in params:
        v = grads[p]
        lo = (v.data_ptr() - base) // es
        out.append((lo, lo + v.numel()))
    return out


class GradBuffer:
    """One persistent f32 buffer holding the gradient of every parameter in the
    reference layout; ``param.grad`` are views into it.  Every backward kernel
    ACCUMULATES into it, so the three branch backwards of a triplet step sum
    in place (no autograd AccumulateGrad traffic), the optimizer sees stable
    pointers, and data-parallel training all-reduces one contiguous buffer.
    k_proj/v_proj weights and biases are adjacent so the fused K|V GEMMs write
    both at once."""

    def __init__(self, model, device):
        self.order = model.grad_order() if hasattr(model, "grad_order") else _module_grad_order(model)
        total = sum(p.numel() for p in self.order)
        self.flat = torch.zeros(total, dtype=torch.float32, device=device)
        self.views = {}
        off = 0
        for p in self.order:
            n = p.numel()
            self.views[id(p)] = self.flat[off:off + n].view(p.shape)
            off += n

    def __getitem__(self, p):
        return self.views[id(p)]

    def attach(self):
        """Make every param.grad a view of the buffer.  If any .grad was reset
        (optimizer.zero_grad(set_to_none=True)) or replaced, start from zero and
        carry over gradients that exist."""
        if all(p.grad is not None and p.grad.data_ptr() == self.views[id(p)].data_ptr() for p in self.order):
            return
        self.flat.zero_()
        for p in self.order:
            v = self.views[id(p)]
            if p.grad is not None:
                v.copy_(p.grad)
            p.grad = v
