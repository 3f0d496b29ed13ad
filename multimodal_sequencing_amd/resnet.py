"""CLIP ModifiedResNet (RN50) visual backbone of the LXRT encoder.

Drop-in for models/CLIP/clip/model.py ModifiedResNet (:10-187: 3-conv stem + avg pool,
anti-aliased Bottlenecks with an avg pool before strided 1x1 convs, AttentionPool2d with the
img_len = 2 pair pooling) and the RN branch of LXRTEncoder.forward (lxrt/modeling.py:1014-1030:
LinearPositionEmbedding + VisualTokenTypeEmbedding, :621-705), with the reference's state-dict
names (BatchNorm running statistics included).

MI355X-first:
  * NHWC activations; 1x1 convolutions are the NT GEMM on the weight as stored, 3x3 ones an
    NHWC im2col (K = 9 C padded to a multiple of 64) + the NT GEMM on a (ky, kx, c)-ordered
    weight copy kept per parameter version; dgrad = GEMM + col2im, wgrad = the TN GEMM;
  * BatchNorm with batch statistics in train mode (deterministic Welford partials), running
    statistics in eval mode, ReLU and the bottleneck's residual add fused into its apply pass;
  * the convolutions run once per UNIQUE image of the batch, not once per pair slot: the
    reference feeds every story image to the backbone 2 (N - 1) times (8 for N = 5, its pair
    batch), and since every image appears equally often, its train-mode batch statistics are
    those of the unique images and the gradients of the copies sum to the gradient of the one
    computation, exactly (the running-variance update uses the reference's element count);
  * the attention pool gathers each pair's two images by index with the reference's
    reshape-before-permute token order (clip/model.py:77) — no copies of the 7 x 7 x 2048 maps.
"""
import math

import torch

from . import _native as N
from . import kernels as K
from .params import Spec, normal, ones, uniform, zeros
from .process_inputs import pairs_generator

STAGE_PLANES = (64, 128, 256, 512)


def _conv_spec(name, cout, cin, k):
    b = 1.0 / math.sqrt(cin * k * k)  # nn.Conv2d default (kaiming_uniform, a = sqrt(5))
    return Spec(name, (cout, cin, k, k), uniform(b), transpose=(k == 1))


def _bn_specs(name, c, zero_gamma=False):
    return [Spec(name + ".weight", (c,), zeros if zero_gamma else ones),
            Spec(name + ".bias", (c,), zeros)]


def rn50_arch(layers=(3, 4, 6, 3), width=64):
    """[(kind, name, dims...)] in forward order: the network as data."""
    stem = [("conv", "conv1", 3, width // 2, 3, 2), ("bn", "bn1", width // 2, True),
            ("conv", "conv2", width // 2, width // 2, 3, 1), ("bn", "bn2", width // 2, True),
            ("conv", "conv3", width // 2, width, 3, 1), ("bn", "bn3", width, True)]
    blocks = []
    inpl = width
    for li, (nb, mult) in enumerate(zip(layers, (1, 2, 4, 8))):
        planes = width * mult
        for bi in range(nb):
            stride = 2 if (li > 0 and bi == 0) else 1
            ds = stride > 1 or inpl != planes * 4
            blocks.append({"name": f"layer{li + 1}.{bi}", "inpl": inpl, "planes": planes,
                           "stride": stride, "downsample": ds})
            inpl = planes * 4
    return stem, blocks


def rn50_specs(prefix, layers=(3, 4, 6, 3), width=64, embed=1024, res=224, std=0.02):
    stem, blocks = rn50_arch(layers, width)
    sp = []
    for kind, name, *d in stem:
        if kind == "conv":
            sp.append(_conv_spec(prefix + name + ".weight", d[1], d[0], d[2]))
        else:
            sp += _bn_specs(prefix + name, d[0])
    for blk in blocks:
        p = prefix + blk["name"] + "."
        inpl, pl = blk["inpl"], blk["planes"]
        sp.append(_conv_spec(p + "conv1.weight", pl, inpl, 1))
        sp += _bn_specs(p + "bn1", pl)
        sp.append(_conv_spec(p + "conv2.weight", pl, pl, 3))
        sp += _bn_specs(p + "bn2", pl)
        sp.append(_conv_spec(p + "conv3.weight", pl * 4, pl, 1))
        sp += _bn_specs(p + "bn3", pl * 4, zero_gamma=True)  # clip/model.py:385-388
        if blk["downsample"]:
            sp.append(_conv_spec(p + "downsample.0.weight", pl * 4, inpl, 1))
            sp += _bn_specs(p + "downsample.1", pl * 4)
    C = width * 32
    g = res // 32
    a = prefix + "attnpool."
    s = C ** -0.5
    sp.append(Spec(a + "positional_embedding", (g * g + 1, C), normal(s)))
    # q | k | v packed (one [3C][C] GEMM operand); state-dict names unchanged
    for n in ("q_proj", "k_proj", "v_proj"):
        sp.append(Spec(a + n + ".weight", (C, C), normal(s), transpose=True, pack="apw"))
    for n in ("q_proj", "k_proj", "v_proj"):
        sp.append(Spec(a + n + ".bias", (C,), zeros, pack="apb"))
    sp.append(Spec(a + "c_proj.weight", (embed, C), normal(s), transpose=True))
    sp.append(Spec(a + "c_proj.bias", (embed,), zeros))
    sp.append(Spec(a + "token_type_embedding.weight", (5, C), normal(std)))  # unused (:62-65)
    return sp


def rn50_attach_order(names):
    """Registration order of the reference's modules: AttentionPool2d creates k_proj before
    q_proj (clip/model.py:60-64), while the packed QKV operand keeps q | k | v in the buffer."""
    k = [n for n in names if ".attnpool.k_proj." in n]
    if not k:
        return names
    rest = [n for n in names if n not in set(k)]
    i = next(j for j, n in enumerate(rest) if ".attnpool.q_proj." in n)
    return rest[:i] + k + rest[i:]


def rn50_buffer_names(prefix, layers=(3, 4, 6, 3), width=64):
    """{bn module name: channels} of every BatchNorm (running stats are buffers)."""
    stem, blocks = rn50_arch(layers, width)
    out = {prefix + n: d[0] for kind, n, *d in stem if kind == "bn"}
    for blk in blocks:
        p = prefix + blk["name"] + "."
        out[p + "bn1"] = blk["planes"]
        out[p + "bn2"] = blk["planes"]
        out[p + "bn3"] = blk["planes"] * 4
        if blk["downsample"]:
            out[p + "downsample.1"] = blk["planes"] * 4
    return out


# ------------------------------------------------------------------------------------------------
class ConvWeights:
    """GEMM operands of a 3x3 conv weight: W [Cout][Kp] in (ky, kx, c) column order and its
    transpose [Kp][Cout], in the compute dtype, rebuilt when the store's weights change."""

    def __init__(self):
        self.cache = {}

    def get(self, store, name, Kp):
        hit = self.cache.get(name)
        if hit is not None and hit[0] == store.version and hit[1] is store.shadow:
            return hit[2], hit[3]
        w = store.f32(name)
        cout, cin, kh, kw = w.shape
        g = torch.zeros(cout, Kp, device=w.device, dtype=store.compute_dtype)
        g[:, :kh * kw * cin] = w.permute(0, 2, 3, 1).reshape(cout, -1).to(store.compute_dtype)
        gt = g.t().contiguous()
        self.cache[name] = (store.version, store.shadow, g, gt)
        return g, gt


def _kp(k):
    return (k + 63) // 64 * 64


class ConvFn(torch.autograd.Function):
    """NHWC conv (bias-free) as GEMMs: x [U][H][W][Cin] -> [U][Ho][Wo][Cout]."""

    @staticmethod
    def forward(ctx, x, anchor, store, name, ks, stride, wcache):
        U, H, W, Cin = x.shape
        w = store.f32(name)
        Cout = w.shape[0]
        pad = (ks - 1) // 2
        Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
        rows = U * Ho * Wo
        if ks == 1 and stride == 1:
            y = K._linear(x.reshape(rows, Cin), store.w(name).view(Cout, Cin))
            Kp = Cin
        else:
            Kp = _kp(ks * ks * Cin)
            cols = torch.empty(rows, Kp, device=x.device, dtype=x.dtype)
            N.conv_im2col(x, ks, stride, pad, Kp, cols)
            Wg, _ = wcache.get(store, name, Kp)
            y = K._linear(cols, Wg)
        ctx.save_for_backward(x)
        ctx.meta = (store, name, ks, stride, pad, Kp, wcache, Ho, Wo)
        return y.view(U, Ho, Wo, Cout)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        store, name, ks, stride, pad, Kp, wcache, Ho, Wo = ctx.meta
        U, H, W, Cin = x.shape
        Cout = dy.shape[-1]
        rows = U * Ho * Wo
        dy2 = dy.contiguous().view(rows, Cout)
        if ks == 1 and stride == 1:
            K._wgrad(dy2, x.reshape(rows, Cin), store.g(name).view(Cout, Cin))
            dx = K._dgrad(dy2, store.wt(name)).view(U, H, W, Cin) if ctx.needs_input_grad[0] \
                else None
            return dx, None, None, None, None, None, None
        cols = torch.empty(rows, Kp, device=x.device, dtype=x.dtype)
        N.conv_im2col(x, ks, stride, pad, Kp, cols)
        gW = torch.zeros(Cout, Kp, device=x.device, dtype=torch.float32)
        K._wgrad(dy2, cols, gW)
        del cols
        store.g(name).add_(gW[:, :ks * ks * Cin].view(Cout, ks, ks, Cin).permute(0, 3, 1, 2))
        dx = None
        if ctx.needs_input_grad[0]:
            _, WgT = wcache.get(store, name, Kp)
            dcols = K._dgrad(dy2, WgT)
            dx = torch.empty_like(x)
            N.conv_col2im(dcols, U, H, W, Cin, ks, stride, pad, Kp, dx)
        return dx, None, None, None, None, None, None


class BatchNormFn(torch.autograd.Function):
    """y = relu?(BN(x) + resid) over the rows of an NHWC tensor."""

    @staticmethod
    def forward(ctx, x, resid, anchor, store, name, bufs, relu, train, n_ref, eps=1e-5,
                momentum=0.1):
        C = x.shape[-1]
        mean = torch.empty(C, device=x.device)
        rstd = torch.empty_like(mean)
        y = torch.empty_like(x)
        rm, rv, nbt = bufs
        N.bn_fwd(x, store.f32(name + ".weight"), store.f32(name + ".bias"),
                 None if resid is None else resid.contiguous(), relu, train, eps, momentum,
                 n_ref, mean, rstd, rm if train else rm, rv, y)
        if train:
            nbt.add_(1)
        ctx.save_for_backward(x, y if relu else None, mean, rstd)
        ctx.meta = (store, name, relu, train, resid is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd = ctx.saved_tensors
        store, name, relu, train, has_res = ctx.meta
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_res else None
        N.bn_bwd(dy.contiguous(), y, x, mean, rstd, store.f32(name + ".weight"), train,
                 store.g(name + ".weight"), store.g(name + ".bias"), dx, dres)
        return dx, dres, None, None, None, None, None, None, None, None, None


class AvgPool2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        U, H, W, C = x.shape
        y = torch.empty(U, H // 2, W // 2, C, device=x.device, dtype=x.dtype)
        N.avgpool2(x.contiguous(), y)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty(ctx.shape, device=dy.device, dtype=dy.dtype)
        N.avgpool2(dy.contiguous(), dx, backward=True)
        return dx


class AttnPoolFn(torch.autograd.Function):
    """AttentionPool2d with img_len = 2 (clip/model.py:73-101) + the visual position / token-type
    embeddings (lxrt:628-705): feats [U][S][C] (unique images, NHWC 7 x 7) -> [P * (2S+1)][C]."""

    @staticmethod
    def forward(ctx, feats, anchor, store, pref, lxrt_pref, pairimg, rolepairs, Nst, heads):
        U, S, C = feats.shape
        P = pairimg.shape[0]
        T2 = 2 * S + 1
        G = int(round(math.sqrt(S)))
        a = pref + "attnpool."
        x = torch.empty(P, T2, C, device=feats.device, dtype=feats.dtype)
        N.attnpool_gather(feats, pairimg, store.f32(a + "positional_embedding"), x)
        x2 = x.view(P * T2, C)
        names = [a + n + ".weight" for n in ("q_proj", "k_proj", "v_proj")]
        bnames = [a + n + ".bias" for n in ("q_proj", "k_proj", "v_proj")]
        qkv = K._linear(x2, store.packed(names, "w"), bias=store.packed(bnames, "f32").view(-1))
        o = torch.empty(P * T2, C, device=x.device, dtype=x.dtype)
        lse = torch.empty(P, heads, T2, device=x.device)
        scale = 1.0 / math.sqrt(C // heads)
        N.attn_fwd(P, T2, heads, qkv, 3 * C, 0, C, 2 * C, None, scale, o, C, lse)
        ao = K._linear(o, store.w(a + "c_proj.weight"), bias=store.f32(a + "c_proj.bias"))
        Ch = ao.shape[-1]
        y = torch.empty(P * T2, 2 * Ch, device=x.device, dtype=x.dtype)
        N.attnpool_out(ao, G, store.f32(lxrt_pref + "visual_pos.x_position_embedding.weight"),
                       store.f32(lxrt_pref + "visual_pos.y_position_embedding.weight"),
                       store.f32(lxrt_pref + "visual_token_type.token_type_embedding.weight"), y)
        ctx.save_for_backward(feats, x2, qkv, o, lse)
        ctx.meta = (store, a, lxrt_pref, names, bnames, rolepairs, Nst, heads, P, T2, G, Ch)
        return y

    @staticmethod
    def backward(ctx, dy):
        feats, x2, qkv, o, lse = ctx.saved_tensors
        store, a, lp, names, bnames, rolepairs, Nst, heads, P, T2, G, Ch = ctx.meta
        U, S, C = feats.shape
        dy = dy.contiguous()
        dao = torch.empty(P * T2, Ch, device=dy.device, dtype=dy.dtype)
        tok = torch.empty(T2, 2 * Ch, device=dy.device)
        N.attnpool_out_bwd(dy, P, T2, Ch, dao, tok)
        # position / token-type gradients from the per-token column sums
        q = torch.arange(T2, device=dy.device)
        grid = torch.where(q == 0, torch.zeros_like(q), (q - 1) % (G * G))
        typ = torch.where(q == 0, torch.zeros_like(q), (q - 1) // (G * G))
        gx = store.g(lp + "visual_pos.x_position_embedding.weight")
        gy = store.g(lp + "visual_pos.y_position_embedding.weight")
        gt = store.g(lp + "visual_token_type.token_type_embedding.weight")
        gx.index_add_(0, grid // G, tok)
        gy.index_add_(0, grid % G, tok)
        gt.index_add_(0, typ, tok)
        K._wgrad(dao, o, store.g(a + "c_proj.weight"), store.g(a + "c_proj.bias"))
        do = K._dgrad(dao, store.wt(a + "c_proj.weight"))
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(P, heads, T2, device=dy.device)
        scale = 1.0 / math.sqrt(C // heads)
        N.attn_bwd(P, T2, heads, qkv, 3 * C, 0, C, 2 * C, None, scale, o, C, do, C, lse, delta,
                   dqkv, 3 * C)
        K._wgrad(dqkv, x2, store.packed(names, "g"), store.packed(bnames, "g").view(-1))
        dx = K._dgrad(dqkv, store.wt(names[0]))
        # positional embedding: every token's gradient at its position (mean token: position 0)
        dxv = dx.view(P, T2, C)
        gpos = store.g(a + "positional_embedding")
        pidx = torch.where(q <= S, q, q - S - 1)
        gpos.index_add_(0, pidx, dxv.float().sum(0))
        dfeats = torch.empty_like(feats)
        N.attnpool_gather_bwd(dx, Nst, rolepairs, dfeats)
        return dfeats, None, None, None, None, None, None, None, None


# ------------------------------------------------------------------------------------------------
class RN50Backbone:
    """Runs the ModifiedResNet of an LXRT store over the unique images of a batch."""

    def __init__(self, store, buffers, prefix, lxrt_prefix="encoder.", layers=(3, 4, 6, 3),
                 width=64, heads=None):
        self.store, self.buffers = store, buffers
        self.prefix, self.lxrt_prefix = prefix, lxrt_prefix
        self.stem, self.blocks = rn50_arch(layers, width)
        self.heads = heads or width * 32 // 64
        self.wcache = ConvWeights()
        self._tables = {}

    def _bn(self, x, name, relu, train, n_ref, anchor, resid=None):
        return BatchNormFn.apply(x, resid, anchor, self.store, name, self.buffers[name], relu,
                                 train, n_ref)

    def _conv(self, x, name, ks, stride, anchor):
        return ConvFn.apply(x, anchor, self.store, name, ks, stride, self.wcache)

    def tables(self, Nst, device):
        if (Nst, device) not in self._tables:
            pairs, _ = pairs_generator(Nst)
            role = [[[] for _ in range(2)] for _ in range(Nst)]
            for j, (a, c) in enumerate(pairs):
                role[a][0].append(j)
                role[c][1].append(j)
            self._tables[(Nst, device)] = torch.tensor(role, dtype=torch.int32, device=device)
        return self._tables[(Nst, device)]

    def forward(self, images, pairs_list, anchor, train, dtype):
        """images [B][N][3][R][R] f32, pairs_list [B][npair][2] -> ([P * T2][2048], T2)."""
        B, Nst = images.shape[:2]
        R = images.shape[-1]
        U = B * Nst
        mult = 2 * (Nst - 1)  # copies of each image in the reference's pair batch
        p = self.prefix
        x = images.reshape(U, 3, R, R).permute(0, 2, 3, 1).to(dtype).contiguous()
        for kind, name, *d in self.stem:
            if kind == "conv":
                x = self._conv(x, p + name + ".weight", d[2], d[3], anchor)
            else:
                x = self._bn(x, p + name, True, train, mult * x.numel() // x.shape[-1], anchor)
        x = AvgPool2Fn.apply(x)
        for blk in self.blocks:
            q = p + blk["name"] + "."
            rows = lambda t: mult * t.numel() // t.shape[-1]  # noqa: E731
            h = self._bn(self._conv(x, q + "conv1.weight", 1, 1, anchor), q + "bn1", True, train,
                         rows(x), anchor)
            h = self._conv(h, q + "conv2.weight", 3, 1, anchor)
            h = self._bn(h, q + "bn2", True, train, rows(h), anchor)
            if blk["stride"] > 1:
                h = AvgPool2Fn.apply(h)
            h = self._conv(h, q + "conv3.weight", 1, 1, anchor)
            if blk["downsample"]:
                idn = AvgPool2Fn.apply(x) if blk["stride"] > 1 else x
                idn = self._conv(idn, q + "downsample.0.weight", 1, 1, anchor)
                idn = self._bn(idn, q + "downsample.1", False, train, rows(idn), anchor)
            else:
                idn = x
            x = self._bn(h, q + "bn3", True, train, rows(h), anchor, resid=idn)
        Ug, G1, G2, C = x.shape
        pl = pairs_list.reshape(B, -1, 2).to(torch.int64)
        base = (torch.arange(B, device=pl.device) * Nst)[:, None, None]
        pairimg = (pl + base).reshape(-1, 2).to(torch.int32).contiguous()
        y = AttnPoolFn.apply(x.reshape(U, G1 * G2, C), anchor, self.store, p, self.lxrt_prefix,
                             pairimg, self.tables(Nst, x.device), Nst, self.heads)
        return y, 2 * G1 * G2 + 1
