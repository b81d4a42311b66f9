"""Device-buffer plumbing for the GPU parity tests (torch only allocates and copies)."""
import ctypes as C

import numpy as np


_KEEP = []


def dev(t, a):
    """numpy -> torch cuda tensor with the same bytes. The tensor is kept alive until release()
    so that an inline `ptr(dev(...))` cannot hand a freed (and reused) block to a kernel."""
    x = _dev(t, a)
    _KEEP.append(x)
    return x


def release():
    _KEEP.clear()


def _dev(t, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.float16 or a.dtype == np.uint16:
        return t.from_numpy(a.view(np.int16).copy()).cuda()
    if a.dtype == np.uint32:
        return t.from_numpy(a.view(np.int32).copy()).cuda()
    if a.dtype == np.uint8:
        return t.from_numpy(a.copy()).cuda()
    if a.dtype == np.uint64:
        return t.from_numpy(a.view(np.int64).copy()).cuda()
    return t.from_numpy(a.copy()).cuda()


def host(x, dtype):
    a = x.detach().cpu().numpy()
    return a.view(dtype)


def ptr(x):
    return C.c_void_p(x.data_ptr() if x is not None else 0)
