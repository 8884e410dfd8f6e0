"""Device ops: HIP kernel entry points of the runtime (copies, page pack/unpack,
managed gather) and the decode-step math used by the models."""
from . import decode  # noqa: F401
from .memory import managed_embedding, ring_copy, gather_pages, scatter_pages  # noqa: F401
