"""yanerf_amd: MI355X-native (gfx950) volumetric-rendering hot path for yet-another-nerf.

Package layout:
  csrc/        HIP kernels + the C ABI (include/yanerf_hip.h) -> libyanerf_hip.so
  _C.py        ctypes binding (raises if the library is missing: there is no CPU fallback)
  ops.py       autograd Functions over the C ABI
  pipelines/   registry-compatible mirror of the reference's yanerf.pipelines (RAY_SAMPLERS / MODELS /
               RENDERERS / PIPELINES with the same class names and signatures)
  parallel.py  one-process-per-GPU data parallelism over torch.distributed (RCCL on ROCm)
  train.py     fused training step (raygen -> coarse/fine MLP -> composite -> loss -> backward -> Adam)
"""
__version__ = "0.1.0"
