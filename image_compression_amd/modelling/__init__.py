"""Drop-in for the reference's `modelling` package (hot path on HIP)."""
from .meta_arch import build_model, META_ARCH_REGISTRY, Compressor2018
from .loss import SSIMLoss, MS_SSIMLoss, MSELoss, get_loss_dict
