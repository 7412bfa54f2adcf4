"""Checkpoint compatibility with the reference.

Reference format (utils/checkpointers/iter_checkpointer.py:49-92): a torch.save
dict {"state_dict": model.state_dict(), <checkpointable>: obj.state_dict()
(optimizer, scheduler), "iter": int, "best_metric": float}, written as
checkpoints/iter_XXXXXXXX.pth (+ iter_XXXXXXXX_<metric>.pth for a new best)
with a rotation log checkpoints/checkpoints_logs.json.  The reference trains
under nn.DataParallel, so its state-dict keys carry a "module." prefix.

* `load_model_weights(model, path_or_dict)` — accepts reference checkpoints
  (prefixed or not, bare state dicts too) and loads with the reference's key
  names; loading never executes pickled code (torch.load weights_only=True).
* `IterCheckpointer` — the reference's save / rotate / resume behaviour and
  file layout; it writes "module."-prefixed keys so the reference can load
  checkpoints trained here.
"""
import collections
import json
import os

import torch

PREFIX = "module."


def strip_prefix(sd, prefix=PREFIX):
    if sd and all(k.startswith(prefix) for k in sd):
        return collections.OrderedDict((k[len(prefix):], v) for k, v in sd.items())
    return sd


def add_prefix(sd, prefix=PREFIX):
    return collections.OrderedDict((k if k.startswith(prefix) else prefix + k, v) for k, v in sd.items())


def load_file(path, map_location="cpu"):
    """torch.load without executing pickled code (weights_only=True)."""
    return torch.load(path, map_location=map_location, weights_only=True)


def load_model_weights(model, src, strict=True):
    """Load reference (or our) weights into `model`; `src` is a path, a
    checkpoint dict with "state_dict", or a bare state dict."""
    cp = load_file(src) if isinstance(src, (str, os.PathLike)) else src
    sd = cp["state_dict"] if isinstance(cp, dict) and "state_dict" in cp else cp
    target = getattr(model, "module", model)
    return target.load_state_dict(strip_prefix(sd), strict=strict)


class IterCheckpointer:
    """reference utils/checkpointers/iter_checkpointer.py:22-162."""

    def __init__(self, folder, model, num_checkpoints=10, logger=None, **checkpointables):
        self.model = model
        self.checkpointables = checkpointables
        self.num_ckpt = int(num_checkpoints)
        self.logger = logger
        self.cp_folder = os.path.join(folder, "checkpoints")
        os.makedirs(self.cp_folder, exist_ok=True)
        self.cp_logs = self._load_cp_log()
        self.additional_info = {"iter": 1, "best_metric": -1.0}

    def _log(self, msg):
        if self.logger is not None:
            self.logger.info(msg)

    def _load_cp_log(self):
        path = os.path.join(self.cp_folder, "checkpoints_logs.json")
        if os.path.isfile(path):
            with open(path) as f:
                logs = json.load(f)
        else:
            logs = {"last_checkpoint": None, "least_recent_checkpoint": None, "best_checkpoint": None,
                    "pretrained": None, "all_checkpoints": []}
        self._all_cps = collections.deque(logs.get("all_checkpoints", []))
        return logs

    def save_checkpoint(self, is_val, **additional_info):
        current_metric = additional_info.pop("current_metric") if is_val else -1.1
        is_best = current_metric > self.additional_info["best_metric"]
        if is_best:
            self._log(f"main metric improve from {self.additional_info['best_metric']} to {current_metric}")
            self.additional_info["best_metric"] = current_metric
        self.additional_info.update(additional_info)
        current_iter = additional_info["iter"]
        model = getattr(self.model, "module", self.model)
        cp = {"state_dict": add_prefix(model.state_dict())}
        for key, ob in self.checkpointables.items():
            cp[key] = ob.state_dict()
        cp.update(self.additional_info)
        path = os.path.join(self.cp_folder, f"iter_{current_iter:0>8}.pth")
        torch.save(cp, path)
        cp_name = ""
        if is_best:
            cp_name = f"iter_{current_iter:0>8}_{current_metric:.4f}.pth"
            torch.save(cp, os.path.join(self.cp_folder, cp_name))
        self._update_cp_log(cp_name)
        return path

    def _update_cp_log(self, best_cp_name):
        cp_name = f"iter_{self.additional_info['iter']:0>8}.pth"
        least = self.cp_logs["least_recent_checkpoint"]
        if least is not None and len(self._all_cps) >= self.num_ckpt:
            p = os.path.join(self.cp_folder, least)
            if os.path.exists(p):
                os.remove(p)
        self._all_cps.append(cp_name)
        self.cp_logs["last_checkpoint"] = cp_name
        idx = max(0, len(self._all_cps) - self.num_ckpt)
        self.cp_logs["least_recent_checkpoint"] = self._all_cps[idx]
        if best_cp_name:
            cur = self.cp_logs["best_checkpoint"]
            if cur and os.path.exists(os.path.join(self.cp_folder, cur)):
                os.remove(os.path.join(self.cp_folder, cur))
            self.cp_logs["best_checkpoint"] = best_cp_name
        if len(self._all_cps) > self.num_ckpt:
            self._all_cps.popleft()
        self.cp_logs["all_checkpoints"] = list(self._all_cps)
        with open(os.path.join(self.cp_folder, "checkpoints_logs.json"), "w") as f:
            json.dump(self.cp_logs, f, indent=4)

    def load_resume(self, pretrained_w=None):
        """Resume from the last checkpoint (returns the next iteration), else
        fine-tune from `pretrained_w`, else start at 1 (iter_checkpointer.py:95-129)."""
        last = self.cp_logs["last_checkpoint"]
        if last is not None:
            cp = load_file(os.path.join(self.cp_folder, last))
            cp["iter"] += 1
            load_model_weights(self.model, cp)
            for key, ob in self.checkpointables.items():
                if key in cp:
                    ob.load_state_dict(cp[key])
            self.additional_info = {k: cp[k] for k in ("iter", "best_metric") if k in cp}
            self._log(f"resume from checkpoint {last}")
            return cp["iter"]
        if pretrained_w is not None:
            load_model_weights(self.model, pretrained_w)
            self.cp_logs["pretrained"] = pretrained_w
            return 1
        return 1
