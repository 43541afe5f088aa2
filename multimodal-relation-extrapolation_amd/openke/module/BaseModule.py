"""BaseModule: checkpoint / parameter I/O of OpenKE modules (OpenKE/openke/module/BaseModule.py:7-55)."""
import json

import torch
import torch.nn as nn


class BaseModule(nn.Module):
    def __init__(self):
        super().__init__()
        self.zero_const = nn.Parameter(torch.Tensor([0]), requires_grad=False)
        self.pi_const = nn.Parameter(torch.Tensor([3.14159265358979323846]), requires_grad=False)

    def load_checkpoint(self, path, map_location=None):
        self.load_state_dict(torch.load(path, map_location=map_location, weights_only=True))
        self.eval()

    def save_checkpoint(self, path):
        torch.save(self.state_dict(), path)

    def load_parameters(self, path):
        with open(path) as f:
            parameters = json.loads(f.read())
        self.set_parameters(parameters)

    def save_parameters(self, path):
        with open(path, "w") as f:
            f.write(json.dumps(self.get_parameters("list")))

    def get_parameters(self, mode="numpy", param_dict=None):
        all_param = self.state_dict()
        keys = all_param.keys() if param_dict is None else param_dict
        res = {}
        for k in keys:
            v = all_param[k]
            res[k] = v.cpu().numpy() if mode == "numpy" else (v.cpu().numpy().tolist() if mode == "list" else v)
        return res

    def set_parameters(self, parameters):
        state = {k: torch.Tensor(v) for k, v in parameters.items()}
        self.load_state_dict(state, strict=False)
        self.eval()
