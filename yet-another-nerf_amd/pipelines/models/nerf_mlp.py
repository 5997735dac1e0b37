"""NeRFMLP on the HIP path (reference yanerf/pipelines/models/nerf_mlp.py).

The module tree (xyz_encoder.mlp.{i}.0, intermediate_linear, density_layer, color_layer.{0,2}) and the
initialisation calls are the reference's, in the same order, so `torch.manual_seed(s); NeRFMLP(**cfg)` draws the
same initial weights and state_dicts/checkpoints interchange with the reference. forward() packs the parameters
into the kernel layout (re-packed only when a parameter changed) and runs the fused PE + MLP + heads kernel; the
backward runs the fused dX kernel + split-K dW kernels (ops._MLPFn)."""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from ... import _C, ops
from .builder import MODELS
from .utils import HarmonicEmbedding, LinearWithRepeat

# bf16: bf16 MFMA with fp8 e4m3 storage of the saved activations / gradient rows (the throughput mode); bf16s: the same
# bf16 MFMA kernels with every stored section bf16 (the precision of the reference under torch.autocast bf16)
_PRECISIONS = {"fp32": _C.PREC_F32, "f32": _C.PREC_F32, "bf16": _C.PREC_BF16, "fp32x3": _C.PREC_F32X3,
               "bf16s": _C.PREC_BF16S}


def _xavier_init(linear) -> None:  # nerf_mlp.py:292-296
    torch.nn.init.xavier_uniform_(linear.weight.data)


class MLPWithInputSkips(torch.nn.Module):
    """Trunk: n_layers x (Linear + ReLU), cat(y, z) before the skip layers (nerf_mlp.py:186-289).
    NOTE the reference builds it with the default hidden_dim=256 (nerf_mlp.py:88-95, 225)."""

    def __init__(self, n_layers: int = 8, input_dim: int = 39, output_dim: int = 256, skip_dim: int = 39,
                 hidden_dim: int = 256, input_skips: List[int] = [5], skip_affine_trans: bool = False,
                 no_last_relu: bool = False):
        super().__init__()
        if skip_affine_trans:
            raise NotImplementedError("skip_affine_trans is not on the HIP path (unused by the reference configs)")
        layers = []
        for li in range(n_layers):
            dimin = hidden_dim if li > 0 else input_dim
            dimout = hidden_dim if li + 1 < n_layers else output_dim
            if li > 0 and li in input_skips:
                dimin = hidden_dim + skip_dim
            linear = torch.nn.Linear(dimin, dimout)
            _xavier_init(linear)
            layers.append(torch.nn.Sequential(linear, torch.nn.ReLU(True))
                          if not no_last_relu or li + 1 < n_layers else linear)
        if no_last_relu:
            raise NotImplementedError("no_last_relu is not on the HIP path (unused by the reference configs)")
        self.mlp = torch.nn.ModuleList(layers)
        self._input_skips = set(input_skips)


@MODELS.register_module()
class NeRFMLP(torch.nn.Module):
    def __init__(
        self,
        n_layers: int = 8,
        input_skips: List[int] = [5],
        n_harmonic_functions_xyz: int = 10,
        harmonic_functions_xyz_append_intput: bool = True,
        n_hidden_neurons_xyz: int = 256,
        n_harmonic_functions_dir: int = 4,
        harmonic_functions_dir_append_intput: bool = True,
        n_hidden_neurons_dir: int = 128,
        latent_dim: int = 0,
        input_xyz: bool = True,
        input_dir: bool = True,
        color_dim: int = 3,
        nerf_paper_v1=False,
        precision: Optional[str] = None,
    ) -> None:
        super().__init__()
        self.n_layers = n_layers
        self.input_skips = list(input_skips)
        self.n_harmonic_functions_xyz = n_harmonic_functions_xyz
        self.harmonic_functions_xyz_append_intput = harmonic_functions_xyz_append_intput
        self.n_hidden_neurons_xyz = n_hidden_neurons_xyz
        self.n_harmonic_functions_dir = n_harmonic_functions_dir
        self.harmonic_functions_dir_append_intput = harmonic_functions_dir_append_intput
        self.n_hidden_neurons_dir = n_hidden_neurons_dir
        self.latent_dim = latent_dim
        self.input_xyz = input_xyz
        self.input_dir = input_dir
        self.color_dim = color_dim
        self.nerf_paper_v1 = nerf_paper_v1
        prec = precision or os.environ.get("YANERF_PRECISION", "fp32")
        if prec not in _PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_PRECISIONS)}, got {prec}")
        self.precision = prec

        self.harmonic_embedding_xyz = HarmonicEmbedding(n_harmonic_functions_xyz,
                                                        append_input=harmonic_functions_xyz_append_intput)
        self.harmonic_embedding_dir = HarmonicEmbedding(n_harmonic_functions_dir,
                                                        append_input=harmonic_functions_dir_append_intput)
        if not input_xyz and latent_dim <= 0:
            raise ValueError("The latent dimension has to be > 0 if xyz is not input!")
        embedding_dim_dir = self.harmonic_embedding_dir.get_output_dim()
        xyz_dim = self.get_xyz_embedding_dim()
        self.xyz_encoder = MLPWithInputSkips(n_layers=n_layers, input_dim=xyz_dim, output_dim=n_hidden_neurons_xyz,
                                             skip_dim=xyz_dim, input_skips=self.input_skips)
        self.intermediate_linear = torch.nn.Linear(n_hidden_neurons_xyz, n_hidden_neurons_xyz)
        _xavier_init(self.intermediate_linear)
        self.density_layer = torch.nn.Linear(n_hidden_neurons_xyz, 1)
        _xavier_init(self.density_layer)
        self.density_layer.bias.data[:] = 0.0
        self.color_layer = torch.nn.Sequential(
            LinearWithRepeat(n_hidden_neurons_xyz + embedding_dim_dir, n_hidden_neurons_dir)
            if input_dir else torch.nn.Linear(n_hidden_neurons_xyz, n_hidden_neurons_dir),
            torch.nn.ReLU(True),
            *([torch.nn.Linear(n_hidden_neurons_dir, n_hidden_neurons_dir), torch.nn.ReLU(True)]
              * ((n_layers // 4) if nerf_paper_v1 else 0)),
            torch.nn.Linear(n_hidden_neurons_dir, color_dim),
            torch.nn.Sigmoid(),
        )
        self._pack_key = None
        self._packed = None

    def get_xyz_embedding_dim(self):
        return self.harmonic_embedding_xyz.get_output_dim() * int(self.input_xyz) + self.latent_dim

    # ------------------------------------------------------------------ HIP path
    def spec(self) -> ops.MlpSpec:
        if not self.input_xyz or not self.input_dir or self.nerf_paper_v1:
            raise NotImplementedError(
                "the HIP NeRFMLP covers input_xyz=True, input_dir=True, nerf_paper_v1=False (every reference "
                "configuration; latent codes are supported)")
        return ops.MlpSpec(n_layers=self.n_layers, input_skips=tuple(self.input_skips),
                           n_harmonic_functions_xyz=self.n_harmonic_functions_xyz,
                           n_harmonic_functions_dir=self.n_harmonic_functions_dir,
                           append_xyz=self.harmonic_functions_xyz_append_intput,
                           append_dir=self.harmonic_functions_dir_append_intput,
                           n_hidden_neurons_xyz=self.n_hidden_neurons_xyz,
                           n_hidden_neurons_dir=self.n_hidden_neurons_dir, color_dim=self.color_dim,
                           precision=_PRECISIONS[self.precision])

    def hip_params(self) -> List[torch.nn.Parameter]:
        """Parameters in the C ABI order (yanerf_mlp_pack)."""
        ps = []
        for layer in self.xyz_encoder.mlp:
            ps += [layer[0].weight, layer[0].bias]
        ps += [self.intermediate_linear.weight, self.intermediate_linear.bias, self.density_layer.weight,
               self.density_layer.bias, self.color_layer[0].weight, self.color_layer[0].bias,
               self.color_layer[-2].weight, self.color_layer[-2].bias]
        return ps

    def packed_weights(self, spec: Optional[ops.MlpSpec] = None) -> torch.Tensor:
        spec = spec or self.spec()
        params = self.hip_params()
        key = (spec.precision,) + tuple((p.data_ptr(), p._version) for p in params)
        if key != self._pack_key:
            # a NEW buffer each time: graphs recorded before an optimizer step keep the weights they used
            self._packed = ops.mlp_pack(spec, params)
            self._pack_key = key
        return self._packed

    def _check_input(self, global_codes) -> bool:  # nerf_mlp.py:179-183
        if global_codes is None:
            return self.latent_dim == 0
        return global_codes.shape[-1] == self.latent_dim

    def _coded_params(self, code: torch.Tensor) -> List[torch.Tensor]:
        """Parameters with a global code folded in. The code is appended to the xyz embedding (embeds = [PE(x),
        code], nerf_mlp.py:299-335) and therefore enters layer 0 and every skip layer ([h, PE(x), code],
        nerf_mlp.py:280-283) through their last latent_dim weight columns; being constant over the batch element's
        points, W[:, code cols] @ code is a bias. The kernel runs with the PE columns only and bias' = b + W_c code;
        autograd carries the bias gradient back to W_c and to the code."""
        ps = []
        for li, layer in enumerate(self.xyz_encoder.mlp):
            w, b = layer[0].weight, layer[0].bias
            if li == 0 or li in self.xyz_encoder._input_skips:
                keep = w.shape[1] - self.latent_dim  # pe (layer 0) or hidden + pe (skip layers)
                b = b + w[:, keep:] @ code
                w = w[:, :keep].contiguous()
            ps += [w, b]
        return ps + self.hip_params()[2 * len(self.xyz_encoder.mlp):]

    def forward(self, origins: torch.Tensor, directions: torch.Tensor, lengths: torch.Tensor,
                global_codes: Optional[torch.Tensor] = None, **kwargs) -> dict:
        """nerf_mlp.py:117-177. global_codes [B, N_latents, latent_dim] (flattened per batch element, :160-161)."""
        if global_codes is not None:
            global_codes = global_codes.view(global_codes.shape[0], -1)
        if not self._check_input(global_codes):
            raise ValueError("The shape of global codes is imcompible with the input dim of the network.")
        spec = self.spec()
        if global_codes is None:
            sigma, rgb = ops.mlp_forward(spec, self.packed_weights(spec), origins, directions, lengths,
                                         self.hip_params())
            return dict(rays_densities=sigma, rays_features=rgb, aux={})
        outs = []
        for b in range(origins.shape[0]):  # one launch per batch element: its code is a per-layer bias
            ps = self._coded_params(global_codes[b].to(origins.dtype))
            outs.append(ops.mlp_forward(spec, ops.mlp_pack(spec, ps), origins[b:b + 1], directions[b:b + 1],
                                        lengths[b:b + 1], ps))
        sigma = torch.cat([o[0] for o in outs], 0)
        rgb = torch.cat([o[1] for o in outs], 0)
        return dict(rays_densities=sigma, rays_features=rgb, aux={})
