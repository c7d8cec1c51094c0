"""ponyc_amd — an MI355X-native actor-dispatch engine for the Pony runtime's
data-parallel hot path (mailbox drain + behaviour dispatch), exposed through the
C-ABI in include/gpu_actor.h and this Python host binding."""
from .engine import Engine, GpuActorError, MSG_DTYPE, load_library  # noqa: F401

__all__ = ["Engine", "GpuActorError", "MSG_DTYPE", "load_library"]
