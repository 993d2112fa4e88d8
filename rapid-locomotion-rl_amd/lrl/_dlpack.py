"""Zero-copy torch views over liblrl device buffers (the gymtorch.wrap_tensor analogue,
legged_robot.py:950-970): an ``lrl_tensor`` descriptor is packed into a DLPack capsule with ctypes
and handed to ``torch.from_dlpack``.  The sim keeps ownership; the capsule has no deleter."""
import ctypes as C

import torch

from . import _abi

kDLROCM = 10


class _DLDevice(C.Structure):
    _fields_ = [("device_type", C.c_int32), ("device_id", C.c_int32)]


class _DLDataType(C.Structure):
    _fields_ = [("code", C.c_uint8), ("bits", C.c_uint8), ("lanes", C.c_uint16)]


class _DLTensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("device", _DLDevice), ("ndim", C.c_int32), ("dtype", _DLDataType),
                ("shape", C.POINTER(C.c_int64)), ("strides", C.POINTER(C.c_int64)), ("byte_offset", C.c_uint64)]


class _DLManagedTensor(C.Structure):
    pass


_DLManagedTensor._fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", C.c_void_p),
                             ("deleter", C.CFUNCTYPE(None, C.POINTER(_DLManagedTensor)))]

_PyCapsule_New = C.pythonapi.PyCapsule_New
_PyCapsule_New.restype = C.py_object
_PyCapsule_New.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p]

_CODE = {0: (2, 32), 1: (0, 32), 2: (1, 8)}  # lrl dtype -> (DLPack code, bits): f32, i32, u8

_keepalive = []  # descriptors must outlive the tensors; sims are few and long-lived


def wrap(desc, device_index):
    """lrl_tensor -> torch.Tensor view (no copy)."""
    nd = desc.ndim
    shape = (C.c_int64 * nd)(*[desc.shape[i] for i in range(nd)])
    strides = (C.c_int64 * nd)(*[desc.strides[i] for i in range(nd)])
    code, bits = _CODE[desc.dtype]
    mt = _DLManagedTensor()
    mt.dl_tensor.data = desc.data
    mt.dl_tensor.device = _DLDevice(kDLROCM, device_index)
    mt.dl_tensor.ndim = nd
    mt.dl_tensor.dtype = _DLDataType(code, bits, 1)
    mt.dl_tensor.shape = shape
    mt.dl_tensor.strides = strides
    mt.dl_tensor.byte_offset = 0
    mt.manager_ctx = None
    mt.deleter = C.cast(None, C.CFUNCTYPE(None, C.POINTER(_DLManagedTensor)))
    _keepalive.append((mt, shape, strides))
    cap = _PyCapsule_New(C.addressof(mt), b"dltensor", None)
    t = torch.from_dlpack(cap)
    if desc.dtype == 2 and t.dtype != torch.uint8:
        t = t.view(torch.uint8)
    return t
