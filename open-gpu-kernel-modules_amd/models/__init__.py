"""Model families running on the tiering runtime."""
from . import llama  # noqa: F401
from .llama import CONFIGS, LlamaConfig, TieredLlama  # noqa: F401
