"""MI355X-native (gfx950) SimPO training path for Janus-Pro (OSPO step 5).

Hand-written CDNA4 HIP kernels behind the C ABI in include/ospo_hip.h
(libospo_hip.so); PyTorch-ROCm supplies device memory, streams and
torch.distributed (RCCL).  See DESIGN.md.
"""
__version__ = "0.1.0"
