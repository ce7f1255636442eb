"""Host entry points of the header-only device string library (csrc/include/locust/
dstring.hpp) -- the same ``__host__ __device__`` functions the map kernel runs on the GPU
(reference util.cu:3-139)."""
from .._native import load

_C = load()

strtok_r_tokens = _C.strtok_r_tokens
itoa = _C.itoa
strcmp = _C.strcmp
pack_key = _C.pack_key
