"""Configuration tree with the reference's key names (utils/config.py:20-133)
for everything the hot path reads, plus YAML merging (safe loader only).
No yacs dependency: CfgNode is a dict with attribute access."""
import copy

import yaml


class CfgNode(dict):
    def __init__(self, init=None):
        super().__init__()
        for k, v in (init or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def __getattr__(self, name):
        if name in self:
            return self[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        self[name] = value

    def clone(self):
        return copy.deepcopy(self)

    def merge_from_dict(self, d, path=""):
        for k, v in d.items():
            if k not in self:
                raise KeyError(f"Non-existent config key: {path}{k}")
            if isinstance(self[k], CfgNode):
                if not isinstance(v, dict):
                    raise ValueError(f"{path}{k} must be a mapping")
                self[k].merge_from_dict(v, path + k + ".")
            else:
                old = self[k]
                if isinstance(old, tuple) and isinstance(v, list):
                    v = tuple(v)
                if isinstance(old, float) and isinstance(v, int) and not isinstance(v, bool):
                    v = float(v)
                self[k] = v

    def merge_from_file(self, path):
        with open(path) as f:
            d = yaml.safe_load(f) or {}
        self.merge_from_dict(d)

    def merge_from_list(self, kv):
        assert len(kv) % 2 == 0
        for key, val in zip(kv[0::2], kv[1::2]):
            node = self
            parts = key.split(".")
            for p in parts[:-1]:
                node = node[p]
            if isinstance(val, str):
                try:
                    val = yaml.safe_load(val)
                except yaml.YAMLError:
                    pass
            node[parts[-1]] = val


_DEFAULTS = {
    "EXPERIMENT": "test", "SEED": 0, "DEBUG": False,
    "DIRS": {"OUTPUTS": "", "EXPERIMENT": "", "TRAIN_DATA": "", "TRAIN_METADATA": "", "VAL_DATA": "", "DATA": ""},
    "DATA": {"IN_CHANNELS": 3, "NUM_WORKERS": 4, "INTERPOLATE": "bilinear", "SIZE": 256,
             "MEAN": [0., 0., 0.], "STD": [1., 1., 1.], "TRAIN_DATASET_NAME": "", "VAL_DATASET_NAME": "",
             "DATALOADER_NAME": "infinite_dataloader"},
    "MODEL": {
        "META_ARCHITECTURE": "Compressor2018", "COMPUTE_DTYPE": "fp32_split",
        "STRIDES": [2, 2, 2, 2], "CONV_KERNEL": 5, "INTER_CHANNELS": 192, "LATENT_CHANNELS": 192,
        "HYPER_PRIOR": {"STRIDES": [1, 2, 2], "KERNELS": [3, 5, 5]},
        "ENTROPY_MODEL": {"DIMS": [3, 3, 3], "INIT_SCALE": 10, "BIN": 1., "PROB_EPS": 1e-10,
                          "CONDITIONAL_MODEL": "LaplacianConditionalModel"},
        "LOSS": {"DISTORTION_LOSS_NAMES": ["MSE"], "DISTORTION_LOSS_WEIGHT": 1., "REDUCTION": "none",
                 "SSIM": {"MAX_VAL": 255., "FILTER_SIZE": 11, "FILTER_SIGMA": 1.5, "K1": 0.01, "K2": 0.03,
                          "LOG_SCALE": False, "EPS": 1e-5},
                 "MS_SSIM_WEIGHTS": [0.0448, 0.2856, 0.3001, 0.2363, 0.1333]},
    },
    "SOLVER": {"USE_ITER": True, "GD_STEPS": 1, "IMS_PER_BATCH": 2, "NUM_CHECKPOINTS": 10,
               "CHECKPOINTER_NAME": "IterCheckpointer", "TRAINER_NAME": "Trainer", "EVALUATOR_NAME": "",
               "MONITOR_NAME": "", "MAIN_METRIC": "", "NUM_EPOCHS": 100, "NUM_ITERS": 1 << 20,
               "SCHEDULER_NAME": "cosine_warmup", "DECAY_EPOCHS": 2.4, "DECAY_RATE": 0.97, "WARMUP_EPOCHS": 1,
               "WARMUP_ITERS": 500, "WARMUP_METHOD": "linear", "WARMUP_FACTOR": 1.0 / 3,
               "WEIGHT_SCHEDULER_NAME": "linear_warmup", "WEIGHT_WARMUP_ITERS": 1, "EPS": 1e-4, "GAMMA": 0.1,
               "STEPS": (30000,), "OPT_NAME": "sgd", "GRAD_CLIP": 0.0, "USE_NESTEROV": False,
               "WEIGHT_DECAY": 0.0005, "WEIGHT_DECAY_BIAS": 0.0, "NUM_COSINE_CYCLE": 0.21875, "MOMENTUM": 0.9,
               "BASE_LR": 0.001, "BIAS_LR_FACTOR": 1.},
    "VAL": {"BATCH_SIZE": 1, "SAVE_PRED": False, "ITER_FREQ": 1 << 10, "SAVE_OUTPUT": False},
}


def get_cfg_defaults():
    """Fresh copy of the defaults (same values as the reference's get_cfg_defaults)."""
    return CfgNode(copy.deepcopy(_DEFAULTS))
