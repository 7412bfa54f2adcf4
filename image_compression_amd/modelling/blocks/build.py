from ...registry import Registry

ENTROPY_MODEL_REGISTRY = Registry("ENTROPY_MODEL")
