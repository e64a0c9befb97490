"""m2amd: MI355X (gfx950) runtime for the m2-tts mel-synthesis + vocoder path.

_lib      ctypes binding of include/m2tts_hip.h (libm2tts_hip.so, built in-tree)
ops       tensor-level wrappers, one per C entry point
runtime   packed per-model handle (HipModel) and its cache
parallel  utterance sharding across GPUs (torch.distributed / RCCL)
"""
__all__ = ["_lib", "ops", "runtime"]
