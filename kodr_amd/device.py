"""Device context: one HIP device + one stream (rlnc_ctx)."""
import ctypes

from . import errors
from ._lib import lib


class Context:
    """Wraps rlnc_ctx_create(device, stream).  ``stream`` may be a raw
    hipStream_t (int) so that work lands on a caller's stream, e.g.
    ``torch.cuda.current_stream().cuda_stream``."""

    def __init__(self, device=0, stream=None):
        h = ctypes.c_void_p()
        errors.check(lib().rlnc_ctx_create(device, ctypes.c_void_p(stream or 0), ctypes.byref(h)))
        self._h = h
        self.device = device
        self.route_min_k = 224

    @property
    def handle(self):
        return self._h

    @property
    def stream(self):
        return lib().rlnc_ctx_stream(self._h)

    def synchronize(self):
        errors.check(lib().rlnc_ctx_synchronize(self._h))

    def elim_stats(self):
        """rlnc_ctx_elim_stats: elimination routes summed over the context's
        decoders (gpu, gpu_retried, host_after_gpu, host)."""
        v = [ctypes.c_size_t() for _ in range(4)]
        errors.check(lib().rlnc_ctx_elim_stats(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("gpu", "gpu_retried", "host_after_gpu", "host"), (x.value for x in v)))

    def set_route_min_k(self, min_k):
        """Single decoders' full batches take the GPU elimination from piece
        count min_k on (rlnc_ctx_set_route_min_k; default 224)."""
        errors.check(lib().rlnc_ctx_set_route_min_k(self._h, int(min_k)))
        self.route_min_k = int(min_k)

    def close(self):
        if self._h:
            lib().rlnc_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- device memory plumbing (for device-resident callers / benches)
    def alloc(self, nbytes):
        p = ctypes.c_void_p()
        errors.check(lib().rlnc_dev_alloc(self._h, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, ptr):
        errors.check(lib().rlnc_dev_free(self._h, ctypes.c_void_p(ptr)))

    def h2d(self, dptr, host):
        import numpy as np
        a = np.ascontiguousarray(host, dtype=np.uint8)
        errors.check(lib().rlnc_memcpy_h2d(self._h, ctypes.c_void_p(dptr),
                                           a.ctypes.data_as(ctypes.c_void_p), a.nbytes))

    def register(self, host):
        """Page-lock a numpy array so the engine DMAs straight from/into it."""
        errors.check(lib().rlnc_host_register(self._h, ctypes.c_void_p(host.ctypes.data), host.nbytes))

    def unregister(self, host):
        errors.check(lib().rlnc_host_unregister(self._h, ctypes.c_void_p(host.ctypes.data)))

    def d2h(self, dptr, nbytes):
        import numpy as np
        out = np.empty(nbytes, dtype=np.uint8)
        errors.check(lib().rlnc_memcpy_d2h(self._h, out.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.c_void_p(dptr), nbytes))
        return out

    def event(self):
        e = ctypes.c_void_p()
        errors.check(lib().rlnc_event_create(self._h, ctypes.byref(e)))
        return e

    def record(self, ev):
        errors.check(lib().rlnc_event_record(self._h, ev))

    def wait(self, ev):
        """this context's stream waits (on the device) for ev, recorded on any context"""
        errors.check(lib().rlnc_ctx_wait_event(self._h, ev))

    @staticmethod
    def elapsed_ms(a, b):
        ms = ctypes.c_float()
        errors.check(lib().rlnc_event_elapsed_ms(a, b, ctypes.byref(ms)))
        return ms.value


_default = {}


def default_context(device=0):
    if device not in _default:
        _default[device] = Context(device)
    return _default[device]


def device_count():
    n = ctypes.c_int(0)
    st = lib().rlnc_device_count(ctypes.byref(n))
    return n.value if st == 0 else 0
