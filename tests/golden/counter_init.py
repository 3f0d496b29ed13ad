"""Counter-based deterministic weights (test infrastructure).

Every parameter is a pure function of (its state-dict key, its flat element index), so golden
fixtures need not store weights: the fixture generator loads these into the reference model,
and the tests load the same values into the product model. The hash is splitmix64 over
(fnv1a(key) + index), mapped to U[-0.5, 0.5); the scale per tensor follows the reference init
rules' magnitudes (normal(0, 0.02) Linear/Embedding: lxrt/modeling.py:1244-1255,
berson/modeling_bert.py:464-474; CLIP class/pos/proj width**-0.5: clip/model.py:250-258;
LSTM U(+-1/sqrt(H)): torch default), with small NON-zero biases and LayerNorm affine
parameters so that every bias / affine path is exercised by parity tests.
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _fnv1a(key: str) -> np.uint64:
    h = 0xCBF29CE484222325
    for ch in key.encode():
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return np.uint64(h)


def _uniform(key: str, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = np.arange(n, dtype=np.uint64) + _fnv1a(key)
        x = x * np.uint64(0x9E3779B97F4A7C15)
        x ^= x >> np.uint64(30)
        x = x * np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x = x * np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return ((x >> np.uint64(40)).astype(np.float64) / float(1 << 24) - 0.5).astype(np.float32)


def _scale(key: str, shape) -> tuple:
    """(scale, offset) for a uniform[-0.5,0.5) draw; std of U[-.5,.5) is 0.2887."""
    leaf = key.rsplit(".", 1)[-1]
    is_ln = ("LayerNorm" in key or "layer_norm" in key or ".ln_" in key or "ln_pre" in key
             or "ln_post" in key)
    if is_ln and leaf == "weight":
        return 0.2, 1.0
    if is_ln and leaf == "bias":
        return 0.1, 0.0
    if leaf in ("class_embedding", "positional_embedding", "proj"):
        width = shape[0] if leaf == "proj" else shape[-1]
        return (width ** -0.5) / 0.2887, 0.0
    # ModifiedResNet (RN50): BatchNorm affine / running statistics near identity, convolution
    # weights with std 1/sqrt(fan_in) so activations keep their scale through 50 layers
    is_bn = ".bn" in key or "downsample.1." in key
    if is_bn and leaf == "weight":
        return 0.4, 1.0
    if leaf == "running_var":
        return 0.4, 1.0
    if leaf == "running_mean":
        return 0.2, 0.0
    if leaf == "num_batches_tracked":
        return 0.0, 0.0
    if leaf == "weight" and len(shape) == 4 and shape[-1] in (1, 3):
        return (1.0 / np.sqrt(shape[1] * shape[2] * shape[3])) / 0.2887, 0.0
    if key.startswith("decoder."):  # nn.LSTM default init U(-1/sqrt(H), 1/sqrt(H))
        h = shape[-1] if "weight" in leaf else shape[0] // 4
        return 2.0 / np.sqrt(h), 0.0
    if leaf.endswith("bias"):
        return 0.02, 0.0
    return 0.02 / 0.2887, 0.0


def counter_state_dict(shapes: dict) -> dict:
    """shapes: {key: tuple} -> {key: float32 ndarray} (deterministic everywhere)."""
    out = {}
    for key, shape in shapes.items():
        n = int(np.prod(shape)) if len(shape) else 1
        s, o = _scale(key, shape)
        out[key] = (_uniform(key, n) * s + o).reshape(shape).astype(np.float32)
    return out
