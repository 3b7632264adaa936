"""Normalizer_ts drop-in (N/cnf/utils/normalize.py:61-120).

On the hot path the '-11' normalise/denormalise pair is fused into the SIREN
kernel (nf_networks.SIRENAutodecoder_film.decode); this class keeps the
reference object (params, method, dim, normalize/denormalize/fit_normalize) for
code that uses it directly.
"""
from __future__ import annotations

import torch


class Normalizer_ts:
    def __init__(self, params=None, method="-11", dim=None):
        self.params = params if params is not None else []
        self.method = method
        self.dim = dim

    def fit_normalize(self, data):
        assert isinstance(data, torch.Tensor)
        if len(self.params) == 0:
            if self.method in ("-11", "01"):
                if self.dim is None:
                    self.params = (torch.max(data), torch.min(data))
                else:
                    self.params = (torch.max(data, dim=self.dim, keepdim=True)[0],
                                   torch.min(data, dim=self.dim, keepdim=True)[0])
            elif self.method == "ms":
                if self.dim is None:
                    self.params = (torch.mean(data), torch.std(data))
                else:
                    self.params = (torch.mean(data, dim=self.dim, keepdim=True),
                                   torch.std(data, dim=self.dim, keepdim=True))
            elif self.method == "none":
                self.params = None
        return self.fnormalize(data, self.params, self.method)

    def normalize(self, new_data):
        return self.fnormalize(new_data, self.params, self.method)

    def denormalize(self, new_data_norm):
        return self.fdenormalize(new_data_norm, self.params, self.method)

    def get_params(self):
        return self.params

    @staticmethod
    def fnormalize(data, params, method):
        if method == "none":
            return data
        p0, p1 = params[0].to(data.device), params[1].to(data.device)
        if method == "-11":
            return (data - p1) / (p0 - p1) * 2 - 1
        if method == "01":
            return (data - p1) / (p0 - p1)
        if method == "ms":
            return (data - p0) / p1
        raise ValueError(method)

    @staticmethod
    def fdenormalize(data_norm, params, method):
        if method == "none":
            return data_norm
        p0, p1 = params[0].to(data_norm.device), params[1].to(data_norm.device)
        if method == "-11":
            return (data_norm + 1) / 2 * (p0 - p1) + p1
        if method == "01":
            return data_norm * (p0 - p1) + p1
        if method == "ms":
            return data_norm * p1 + p0
        raise ValueError(method)
