"""Child process of tests/test_io.py::test_readers_survive_corrupted_metadata:
loads one (possibly corrupted) data directory with the product's readers and
prints the return codes.  A crash (signal) of this process is what the test
catches; return codes other than 0 / CLOUDSC_EIO are failures too."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dwarf-p-cloudsc_amd"))
import cloudsc_amd as ca  # noqa: E402  (the Params mirror only; no GPU library is loaded)

IO_LIB = os.environ.get("CLOUDSC_IO_LIB", os.path.join(REPO, "dwarf-p-cloudsc_amd", "libcloudsc_io.so"))   # e.g. a sanitizer build
NIN = 28


class Dataset(C.Structure):   # mirror of cloudsc_dataset_t (tests/test_io.py)
    _fields_ = [("klon", C.c_int), ("klev", C.c_int), ("params", ca.Params),
                ("inp", C.POINTER(C.c_double) * NIN), ("ktype", C.POINTER(C.c_int)),
                ("ref", C.POINTER(C.c_double) * 21), ("has_reference", C.c_int), ("source", C.c_char * 512)]


def main(path):
    lib = C.CDLL(IO_LIB)
    names = ("cloudsc_io_load_serialbox", "cloudsc_io_load_raw", "cloudsc_io_load_dir")
    for fn in names:
        getattr(lib, fn).argtypes = [C.c_char_p, C.c_int, C.POINTER(Dataset)]
    lib.cloudsc_io_free.argtypes = [C.POINTER(Dataset)]
    rcs = []
    for fn in names:
        d = Dataset()
        rc = getattr(lib, fn)(path.encode(), 1, C.byref(d))
        if rc == 0:
            lib.cloudsc_io_free(C.byref(d))
        rcs.append(rc)
    print(" ".join(str(r) for r in rcs))


def main_hdf5(inp, ref):
    lib = C.CDLL(IO_LIB)
    lib.cloudsc_io_load_hdf5.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(Dataset)]
    lib.cloudsc_io_free.argtypes = [C.POINTER(Dataset)]
    d = Dataset()
    rc = lib.cloudsc_io_load_hdf5(inp.encode(), ref.encode() if ref else None, C.byref(d))
    if rc == 0:
        lib.cloudsc_io_free(C.byref(d))
    print(rc)


if __name__ == "__main__":
    if sys.argv[1] == "--hdf5":
        main_hdf5(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        main(sys.argv[1])
