"""bf16 rounding-placement emulation of the encoder — TEST INFRASTRUCTURE ONLY.

The oracle's functional restatement (oracle/berson_oracle.py, which reproduces the reference to
1e-5) run in fp32 on the GPU, with an explicit bf16 rounding r(t) = fp32(bf16(t)) inserted at
chosen SITES of the encoder. It answers "how large is the error of bf16 arithmetic placed like
this?", independently of the HIP kernels:

  operand  GEMM activation operands rounded to bf16, fp32 accumulation
  weight   GEMM weight operands rounded to bf16
  output   op outputs that feed the next op: QKV, attention output, (Quick)GELU output, the ViT's
           pre-LN block inputs, ViT projection
  prob     attention probabilities rounded before the P.V product (flash attention's bf16 P)
  stream   the residual stream: the ViT's x after every residual add, the BERT layers' pre-LN
           sums and LayerNorm outputs, the embedding / visn_fc / ln_pre outputs
  mx       (not in ALL) the four GEMMs of every encoder layer (QKV, attention output, FC1, FC2) take
           both operands through OCP MX-fp8 quantisation — e4m3 elements, one E8M0 power-of-two
           scale 2^(floor(log2 amax) - 8) per 32 K-elements — after the bf16 rounding, as
           kernels.fp8_forward() does (fp32 accumulation of the dequantised values)

ALL = every site is where the product's bf16 mode rounds (kernels.py / the csrc epilogues).
Follows oracle vit_forward / bert_layer / lxrt_forward (clip/model.py:242-305,
lxrt/modeling.py:496-507,1513-1598) with the rounding added.
"""
import math

import torch
import torch.nn.functional as F

from oracle import berson_oracle as O

ALL = frozenset(("operand", "weight", "output", "prob", "stream"))


def _r(t):
    return t.to(torch.bfloat16).float()


def mx_fake_quant(t):
    """t [..., K] -> its MX-fp8 value (dequantised, fp32): per 32 consecutive K-elements the shared
    exponent e = floor(log2 amax) - 8 (E8M0, clamped to [-127, 127]; all-zero blocks -> 2^-127),
    elements t / 2^e clamped to +-448 and rounded to float8_e4m3fn (csrc/fp8.hip mmseq_quant_mxfp8)."""
    shp = t.shape
    b = t.float().reshape(-1, shp[-1] // 32, 32)
    amax = b.abs().amax(-1, keepdim=True)
    e = torch.where(amax > 0, ((amax.view(torch.int32) >> 23) & 0xFF).float() - 127,
                    torch.full_like(amax, -127.0))
    e = torch.clamp(e - 8, -127, 127)
    s = torch.where(amax > 0, torch.exp2(e), torch.ones_like(e))
    return (torch.clamp(b / s, -448, 448).to(torch.float8_e4m3fn).float() * s).reshape(shp)


class Emu:
    def __init__(self, p, sites):
        self.p = p
        self.s = frozenset(sites)
        self._w = {}

    def rnd(self, site, t):
        return _r(t) if site in self.s else t

    def w(self, name):
        if "weight" not in self.s:
            return self.p[name]
        if name not in self._w:
            self._w[name] = _r(self.p[name])
        return self._w[name]

    def mm(self, x, wkey, mx=False):
        """x @ W^T with the operand / weight rounding (and MX-fp8 quantisation for the layer GEMMs)"""
        x, w = self.rnd("operand", x), self.w(wkey)
        if mx and "mx" in self.s:
            if ("mx", wkey) not in self._w:
                self._w[("mx", wkey)] = mx_fake_quant(w)
            x, w = mx_fake_quant(x), self._w[("mx", wkey)]
        return x @ w.t()

    def lin(self, x, name, bias=True, mx=False):
        y = self.mm(x, name + ".weight", mx)
        if bias and (name + ".bias") in self.p:
            y = y + self.p[name + ".bias"]
        return y

    def ln(self, x, name, eps):
        return F.layer_norm(x, (x.shape[-1],), self.p[name + ".weight"], self.p[name + ".bias"], eps)

    def mha(self, q, k, v, heads, key_bias=None):
        B, T, D = q.shape
        d = D // heads
        qh, kh, vh = (self.rnd("output", t).view(B, t.shape[1], heads, d).transpose(1, 2)
                      for t in (q, k, v))
        s = qh @ kh.transpose(-1, -2) / math.sqrt(d)
        if key_bias is not None:
            s = s + key_bias[:, None, None, :]
        a = self.rnd("prob", torch.softmax(s, -1))
        return self.rnd("output", (a @ vh).transpose(1, 2).reshape(B, T, D))

    def vit(self, images, img_len=2, heads=None):
        p, V = self.p, O.VIT
        w = p[V + "conv1.weight"]
        W, _, ps, _ = w.shape
        heads = heads or W // 64
        x = F.conv2d(self.rnd("operand", images), self.w(V + "conv1.weight"), stride=ps)
        npatch = x.shape[2] * x.shape[3]
        x = x.reshape(x.shape[0], W, -1).permute(0, 2, 1)
        Pn = x.shape[0] // img_len
        x = x.reshape(Pn, -1, W)
        cls = p[V + "class_embedding"] + torch.zeros(Pn, 1, W, device=x.device)
        x = torch.cat([cls, x], 1)
        pos = p[V + "positional_embedding"]
        pos = torch.cat([pos] + [pos[:npatch]] * (img_len - 1), 0)
        x = self.rnd("stream", self.ln(x + pos, V + "ln_pre", 1e-5))
        nl = len({k.split(".")[6] for k in p if k.startswith(V + "transformer.resblocks.")})
        for i in range(nl):
            b = f"{V}transformer.resblocks.{i}."
            h = self.rnd("output", self.ln(x, b + "ln_1", 1e-5))
            qkv = self.mm(h, b + "attn.in_proj_weight", True) + p[b + "attn.in_proj_bias"]
            q, k, v = qkv.split(W, -1)
            x = self.rnd("stream", x + self.lin(self.mha(q, k, v, heads), b + "attn.out_proj", mx=True))
            h = self.rnd("output", self.ln(x, b + "ln_2", 1e-5))
            f = self.rnd("output", O.quick_gelu(self.lin(h, b + "mlp.c_fc", mx=True)))
            x = self.rnd("stream", x + self.lin(f, b + "mlp.c_proj", mx=True))
        return self.rnd("output", self.rnd("operand", x) @ self.w(V + "proj"))

    def bert_layer(self, i, x, key_bias, heads):
        b = f"bert.encoder.layer.{i}."
        q = self.lin(x, b + "attention.self.query", mx=True)
        k = self.lin(x, b + "attention.self.key", mx=True)
        v = self.lin(x, b + "attention.self.value", mx=True)
        a = self.mha(q, k, v, heads, key_bias)
        s = self.rnd("stream", self.lin(a, b + "attention.output.dense", mx=True) + x)
        h = self.rnd("stream", self.ln(s, b + "attention.output.LayerNorm", 1e-12))
        f = self.rnd("output", O.gelu_erf(self.lin(h, b + "intermediate.dense", mx=True)))
        s = self.rnd("stream", self.lin(f, b + "output.dense", mx=True) + h)
        return self.rnd("stream", self.ln(s, b + "output.LayerNorm", 1e-12))

    def lxrt(self, ids, mask, tt, images, heads, vit_heads):
        p = self.p
        ext = (1.0 - mask.float()) * -10000.0
        lang = self.rnd("stream", O.bert_embeddings(p, ids, tt))
        vis = self.vit(images, 2, vit_heads)
        vis = self.rnd("stream", self.ln(self.lin(vis, "bert.encoder.visn_fc.visn_fc"),
                                         "bert.encoder.visn_fc.visn_layer_norm", 1e-12))
        joint = torch.cat([lang, vis], 1)
        key_bias = torch.cat([ext, torch.zeros(vis.shape[0], vis.shape[1], device=ext.device)], 1)
        nl = len({k.split(".")[3] for k in p if k.startswith("bert.encoder.layer.")})
        for i in range(nl):
            joint = self.bert_layer(i, joint, key_bias, heads)
        return joint[:, :ids.shape[1]]


def encode(p, pair, images, cfg, sites):
    """oracle.encode with the emulated encoder (the BERSON head in fp32, as the oracle)."""
    lxrt = O.lxrt_forward
    emu = Emu(p, sites)

    def patched(p_, ids, msk, tt, img, heads, img_len, vit_heads):
        return emu.lxrt(ids, msk, tt, img, heads, vit_heads), None
    O.lxrt_forward = patched
    try:
        return O.encode(p, pair, images, cfg)
    finally:
        O.lxrt_forward = lxrt


def order_nll(p, enc, input_ids, order, n):
    """Pointer NLL of `order` (= beam score: l_ptr x (N - 1)) given a cached encode()."""
    pair = O.prepare_berson_inputs(input_ids, [list(order)], n)
    loss, _ = O.pointer_forward(p, enc, pair, lam=0.0)
    return float(loss) * (n - 1)
