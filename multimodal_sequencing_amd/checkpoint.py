"""Checkpoint interop with the reference (SURVEY §8f row 4, §5 checkpoint/resume).

A checkpoint directory is what the reference writes and reads:
  config.json        the JSON config (lxrt BertConfig / berson BertConfig; sorted keys, indent 2)
  pytorch_model.bin  torch.save(model.state_dict()) with the reference's key names (App. B)
  optimizer.pt       transformers AdamW state (train.py:411-413, resumed at :193-201)
  scheduler.pt       LambdaLR state
so a model trained here loads in the reference and a reference checkpoint (or a pretrained
roberta-large / bert-base directory) loads here.

Loading follows the two loaders the path uses:
  * lxrt BertPreTrainedModel.from_pretrained (models/CLIP/src/lxrt/modeling.py:1258-1433):
    gamma/beta -> weight/bias (:1341-1354); start prefix 'bert.' or 'roberta.' when the model has
    no `.bert` (:1373-1376); for a model WITH `.bert` and a roberta state dict, lm_head.* ->
    cls.predictions.* and roberta -> bert (:1378-1401); missing / unexpected keys are logged,
    shape errors raise (:1422-1431);
  * berson PreTrainedModel.from_pretrained (models/berson/modeling_utils.py:208-428): the same
    gamma/beta rename, then base_model_prefix 'bert' logic (:395-402): a base-model state dict
    loads into `model.bert`, a derived one into the model; eval mode afterwards (:421).

Serialized files are read with torch.load(weights_only=True) only (tensors and plain
containers; nothing in the file is executed).
"""
import json
import logging
import os
import tarfile
import tempfile
import shutil
from collections import OrderedDict

import torch

logger = logging.getLogger(__name__)

CONFIG_NAME = "config.json"  # lxrt/modeling.py CONFIG_NAME, berson/file_utils.py:73
WEIGHTS_NAME = "pytorch_model.bin"  # lxrt/modeling.py:1449, berson/file_utils.py:70
OPTIMIZER_NAME = "optimizer.pt"  # trainers/train.py:411
SCHEDULER_NAME = "scheduler.pt"  # trainers/train.py:413


# ------------------------------------------------------------------------------------------------
# configs
def _jsonable(v):
    try:
        json.dumps(v)
        return True
    except (TypeError, ValueError):
        return False


class JsonConfigMixin:
    """to_json_string / save_pretrained / from_json_file / from_pretrained of the reference's
    config classes (lxrt/modeling.py:213-336, berson/configuration_utils.py:60-190) for a
    SimpleNamespace-style config."""

    def to_dict(self):
        return {k: v for k, v in vars(self).items() if not k.startswith("_") and _jsonable(v)}

    def to_json_string(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True) + "\n"

    def to_json_file(self, path):
        with open(path, "w", encoding="utf-8") as f:
            f.write(self.to_json_string())

    def save_pretrained(self, save_directory):
        assert os.path.isdir(save_directory), \
            "Saving path should be a directory where the model and configuration can be saved"
        self.to_json_file(os.path.join(save_directory, CONFIG_NAME))

    @classmethod
    def from_dict(cls, d):
        cfg = cls()
        for k, v in d.items():
            setattr(cfg, k, v)
        return cfg

    @classmethod
    def from_json_file(cls, path):
        with open(path, "r", encoding="utf-8") as f:
            return cls.from_dict(json.loads(f.read()))

    @classmethod
    def from_pretrained(cls, path, return_unused_kwargs=False, **kwargs):
        """berson configuration_utils.py:73-159: config.json of a directory (or a json file);
        kwargs naming an existing attribute override it, the rest are returned if asked."""
        f = os.path.join(path, CONFIG_NAME) if os.path.isdir(path) else path
        if not os.path.isfile(f):
            raise EnvironmentError(f"no {CONFIG_NAME} at '{path}' (no model-name downloads here)")
        cfg = cls.from_json_file(f)
        if isinstance(getattr(cfg, "pruned_heads", None), dict):
            cfg.pruned_heads = {int(k): set(v) for k, v in cfg.pruned_heads.items()}
        unused = {}
        for k, v in kwargs.items():
            if hasattr(cfg, k):
                setattr(cfg, k, v)
            else:
                unused[k] = v
        return (cfg, unused) if return_unused_kwargs else cfg


# ------------------------------------------------------------------------------------------------
# state dicts
def load_weights_file(path, map_location="cpu"):
    """A pytorch_model.bin / optimizer.pt written by torch.save, tensors and plain containers
    only (weights_only=True: a file needing arbitrary unpickling is refused)."""
    return torch.load(path, map_location=map_location, weights_only=True)


def rename_gamma_beta(state_dict):
    """Old TF-style LayerNorm names: 'gamma' -> 'weight', 'beta' -> 'bias' (lxrt:1341-1354,
    berson modeling_utils.py:365-376). In place, returns the dict."""
    renames = []
    for k in list(state_dict.keys()):
        new = None
        if "gamma" in k:
            new = k.replace("gamma", "weight")
        if "beta" in k:
            new = k.replace("beta", "bias")
        if new:
            renames.append((k, new))
    for old, new in renames:
        state_dict[new] = state_dict.pop(old)
    return state_dict


def roberta_to_bert_keys(state_dict, model_keys):
    """lxrt:1378-1401: a RoBERTa (masked-LM) state dict into a model that has `.bert` and
    BertPreTrainingHeads: lm_head.* -> cls.predictions.*, every other key roberta -> bert. Every
    renamed key must exist in the model (the reference asserts it)."""
    renames = []
    for k in list(state_dict.keys()):
        if k == "lm_head.bias":
            new = "cls.predictions.bias"
        elif "lm_head.dense" in k:
            new = k.replace("lm_head.dense", "cls.predictions.transform.dense")
        elif "lm_head.layer_norm" in k:
            new = k.replace("lm_head.layer_norm", "cls.predictions.transform.LayerNorm")
        elif "lm_head.decoder" in k:
            new = k.replace("lm_head.decoder", "cls.predictions.decoder")
        else:
            new = k.replace("roberta", "bert")
        if new not in model_keys:
            raise KeyError(f"checkpoint key {k!r} -> {new!r} is not a parameter of the model")
        renames.append((k, new))
    for old, new in renames:
        state_dict[new] = state_dict.pop(old)
    return state_dict


class LoadInfo(dict):
    """{'missing_keys', 'unexpected_keys', 'error_msgs'} (berson modeling_utils.py:423-425)."""


def load_into(module, state_dict, prefix=""):
    """Copy `state_dict` into `module` the way the reference's recursive `load(module, prefix)`
    does (_load_from_state_dict with strict bookkeeping): keys under `prefix` are matched after
    stripping it, keys outside it are ignored, missing / unexpected keys are collected and a
    shape mismatch raises. The module's load_state_dict post-hooks mark the bf16 shadows stale."""
    own = module.state_dict(keep_vars=True)
    sub = OrderedDict()
    unexpected = []
    for k, v in state_dict.items():
        if not k.startswith(prefix):
            continue
        kk = k[len(prefix):]
        if kk in own:
            sub[kk] = v
        else:
            unexpected.append(k)
    errors = []
    for kk, v in sub.items():
        if tuple(own[kk].shape) != tuple(v.shape):
            errors.append(f"size mismatch for {kk}: copying a param with shape "
                          f"{tuple(v.shape)} from checkpoint, the shape in current model is "
                          f"{tuple(own[kk].shape)}.")
    if errors:
        raise RuntimeError("Error(s) in loading state_dict for {}:\n\t{}".format(
            type(module).__name__, "\n\t".join(errors)))
    res = module.load_state_dict(sub, strict=False)
    missing = [k for k in res.missing_keys]
    if missing:
        logger.info("Weights of %s not initialized from pretrained model: %s",
                    type(module).__name__, missing)
    if unexpected:
        logger.info("Weights from pretrained model not used in %s: %s",
                    type(module).__name__, unexpected)
    return LoadInfo(missing_keys=missing, unexpected_keys=unexpected, error_msgs=[])


def state_dict_for_save(module):
    """module.state_dict() as standalone CPU tensors: each parameter gets its own storage (they
    are views of one flat device buffer here), tied parameters stay tied (one storage)."""
    out = OrderedDict()
    memo = {}
    for k, v in module.state_dict().items():
        key = (v.data_ptr(), tuple(v.shape), tuple(v.stride()), v.dtype)
        if key not in memo:
            memo[key] = v.detach().to("cpu", copy=True).contiguous()
        out[k] = memo[key]
    return out


def save_pretrained(model, save_directory):
    """lxrt/modeling.py:1435-1453 and berson modeling_utils.py:190-204: config.json +
    pytorch_model.bin in an existing directory."""
    assert os.path.isdir(save_directory), \
        "Saving path should be a directory where the model and configuration can be saved"
    m = model.module if hasattr(model, "module") else model
    m.config.save_pretrained(save_directory)
    out = os.path.join(save_directory, WEIGHTS_NAME)
    torch.save(state_dict_for_save(m), out)
    logger.info("Model weights saved in %s", out)
    return out


def _resolve_dir(path):
    """A checkpoint directory, or a .tar.gz archive of one (lxrt:1319-1329) extracted to a temp
    dir (returned second, for cleanup). Model names needing a download are not resolvable."""
    if os.path.isdir(path):
        return path, None
    if os.path.isfile(path) and tarfile.is_tarfile(path):
        tmp = tempfile.mkdtemp()
        with tarfile.open(path, "r:*") as ar:
            try:
                ar.extractall(tmp, filter="data")
            except TypeError:  # interpreter without extraction filters
                for m in ar.getmembers():
                    if m.name.startswith(("/", "..")) or ".." in m.name.split("/") or \
                            m.issym() or m.islnk() or not (m.isfile() or m.isdir()):
                        raise ValueError(f"unsafe member {m.name!r} in {path}")
                ar.extractall(tmp)
        return tmp, tmp
    raise EnvironmentError(f"'{path}' is not a checkpoint directory or archive "
                           "(pretrained-model names need a download, which is not available)")


def lxrt_from_pretrained(cls, pretrained_model_name_or_path, state_dict=None, cache_dir=None,
                         from_tf=False, *inputs, **kwargs):
    """lxrt BertPreTrainedModel.from_pretrained (:1258-1433) for LXRTModel / LXRTPretraining:
    config.json -> cls(config, *inputs, **kwargs) -> remapped pytorch_model.bin."""
    if from_tf:
        raise NotImplementedError("TensorFlow checkpoints are not supported")
    from .lxrt import LXRTConfig
    d, tmp = _resolve_dir(pretrained_model_name_or_path)
    try:
        config = LXRTConfig.from_json_file(os.path.join(d, CONFIG_NAME))
        model = cls(config, *inputs, **kwargs)
        if state_dict is None:
            state_dict = load_weights_file(os.path.join(d, WEIGHTS_NAME))
    finally:
        if tmp:
            shutil.rmtree(tmp)
    state_dict = rename_gamma_beta(OrderedDict(state_dict))
    has_bert = hasattr(model, "bert")
    prefix = ""
    if not has_bert and any(k.startswith("bert.") for k in state_dict):
        prefix = "bert."
    elif not has_bert and any(k.startswith("roberta.") for k in state_dict):
        prefix = "roberta."
    elif has_bert and any(k.startswith("roberta.") for k in state_dict):
        state_dict = roberta_to_bert_keys(state_dict, set(model.state_dict().keys()))
    model.loading_info = load_into(model, state_dict, prefix)
    return model


def berson_from_pretrained(cls, pretrained_model_name_or_path, *model_args, **kwargs):
    """berson PreTrainedModel.from_pretrained (modeling_utils.py:208-428) for BertForOrdering:
    called as in trainers/train.py:2030-2035 / :2194-2199 with config=, inner_model=,
    tokenizer=, load_inner_model=True, args=."""
    config = kwargs.pop("config", None)
    state_dict = kwargs.pop("state_dict", None)
    output_loading_info = kwargs.pop("output_loading_info", False)
    if kwargs.pop("from_tf", False):
        raise NotImplementedError("TensorFlow checkpoints are not supported")
    for k in ("cache_dir", "force_download", "proxies"):
        kwargs.pop(k, None)
    d, tmp = _resolve_dir(pretrained_model_name_or_path)
    try:
        if config is None:
            from .berson import BersonConfig
            config, kwargs = BersonConfig.from_pretrained(d, return_unused_kwargs=True, **kwargs)
        model = cls(config, *model_args, **kwargs)
        if state_dict is None:
            state_dict = load_weights_file(os.path.join(d, WEIGHTS_NAME))
    finally:
        if tmp:
            shutil.rmtree(tmp)
    state_dict = rename_gamma_beta(OrderedDict(state_dict))
    base = cls.base_model_prefix
    prefix, target = "", model
    if not hasattr(model, base) and any(k.startswith(base) for k in state_dict):
        prefix = base + "."
    if hasattr(model, base) and not any(k.startswith(base) for k in state_dict):
        target = getattr(model, base)
        if target is None:  # the reference would build a BertModel here (modeling_bert.py:860-866)
            raise ValueError(f"state dict has no '{base}.' keys and the model has no inner "
                             f"'{base}' module to load them into: pass inner_model=")
    info = load_into(target, state_dict, prefix)
    model.eval()
    model.loading_info = info
    return (model, info) if output_loading_info else model


# ------------------------------------------------------------------------------------------------
def load_clip_visual_weights(model, weights):
    """trainers/train.py:1885-1897 (--clip_visual_model_weights): every key containing 'visual'
    is loaded into the model, with its first component dropped unless that is 'encoder' (so a
    'bert.encoder.visual_model.visual.*' or 'module.encoder....' file maps onto the model's
    'encoder.visual_model.visual.*'); strict=False."""
    sd = load_weights_file(weights) if isinstance(weights, str) else weights
    own = set(model.state_dict().keys())
    picked = OrderedDict()
    for k, v in sd.items():
        if "visual" not in k:
            continue
        parts = k.split(".")
        name = k if parts[0] == "encoder" else ".".join(parts[1:])
        if name not in own:
            raise KeyError(f"visual weight {k!r} -> {name!r} is not a parameter of the model")
        picked[name] = v
    return model.load_state_dict(picked, strict=False)
