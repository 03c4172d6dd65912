"""The C-ABI boundary on a machine without a GPU: libfrhip.so loads, exports every function
include/frhip.h declares, and rejects bad arguments with FR_ERR_* codes + a message (no compute)."""
import ctypes

from facerecognition_amd import _native as N


def test_library_exports_every_header_symbol():
    L = N.lib()
    names = N.header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(N._SIGS) >= set(names), set(names) - set(N._SIGS)


def test_abi_version():
    assert N.lib().fr_abi_version() == 1


def test_bad_arguments_are_rejected_with_message():
    L = N.lib()
    h = ctypes.c_void_p()
    rc = L.fr_create(ctypes.byref(h), 0, 99, 0)  # unknown arch
    assert rc == -1 and b"arch" in L.fr_last_error()
    rc = L.fr_topk_merge(None, None, 1, 1, 5, None, None, None)
    assert rc == -1 and b"fr_topk_merge" in L.fr_last_error()
    rc = L.fr_topk_merge(None, None, 1, 1, 17, None, None, None)  # k > 16
    assert rc == -1
    rc = L.fr_topk_merge_ranks(None, 2, 1, 5, None, None, None)
    assert rc == -1 and b"fr_topk_merge_ranks" in L.fr_last_error()
    d = N.FrConvDesc()
    assert L.fr_op_conv2d(ctypes.byref(d), None) == -1
    assert b"fr_op_conv2d" in L.fr_last_error()


def test_python_check_raises_with_message():
    L = N.lib()
    L.fr_op_avgpool(None, 1, 1, 1, 8, None, 0, None)
    try:
        N.check(-1, "fr_op_avgpool")
    except RuntimeError as e:
        assert "fr_op_avgpool" in str(e)
    else:
        raise AssertionError("check() did not raise")


def test_weight_blob_round_trip_format():
    import numpy as np
    from facerecognition_amd.weights import pack_blob
    blob = pack_blob({"a.w": np.arange(6, dtype=np.float32).reshape(2, 3), "b": np.zeros(0, np.float32)})
    assert blob[:4] == b"FRW1"
    assert int.from_bytes(blob[4:8], "little") == 2
