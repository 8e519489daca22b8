"""diplomjourney_amd — MI355X-native MPC candidate expansion.

Drop-in for the hot path of ShittyWizard/DiplomJourney (math_model_tree.py
predictive_control): HIP/CDNA4 rollout + cost + arg-min kernels behind a C ABI
(include/mpc_rollout.h), a PyTorch-ROCm host mirroring the reference's
config / CoordinateTree / predictive_control / run_math_model surface, and a
torch.distributed (RCCL) candidate-sharded exchange for multi-GPU.
"""
__version__ = "0.1.0"
