"""MI355X-native multimodal-LLM pre-training step (ViT → projector → Pythia).

Drop-in for the hot path of tttyuntian/multimodal_llm_pretraining: the
per-step forward/backward/optimizer work runs in hand-written HIP kernels for
gfx950 (libmmpt.so, C-ABI in include/mmpt.h); PyTorch-ROCm supplies device
memory, streams and torch.distributed (RCCL) only.
"""

__version__ = "0.1.0"
