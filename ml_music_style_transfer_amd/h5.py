"""HDF5 datasets through the HDF5 C library (ctypes), for the reference's on-disk schema.

The reference stores its training data with h5py (preprocessing/utils/io_manager.py:39-76):
one file per split (`<data_dir>_train.hdf5`, `_test.hdf5`) holding resizable float64
datasets created with `chunks=True, maxshape=(None, ...)` and appended along axis 0:

    pianoroll   (N, T, 128)     onoff   (N, T, 128)     spec_<style>   (N, 1025, T)

and reads them back with `h5py.File(path, 'r')[name][:n_read]` (train.py:47-72).
h5py is not importable in this image, but libhdf5 (1.10, /opt/conda/lib) is; this module
binds the handful of C entry points that reading and appending need. `File` mirrors the
small h5py surface the reference uses: `keys()`, `in`, `[name].shape`, `[name][:n]` /
`[name][a:b]`, `create_dataset(name, data=, dtype='float64', maxshape=(None, ...),
chunks=True)`, `resize(n, axis=0)` and `[name][-k:] = x`. Reads convert to float64 in
the library (H5T_NATIVE_DOUBLE) like h5py does for a float64 dataset.
"""
import ctypes
import ctypes.util
import os

import numpy as np

__all__ = ["File", "Dataset", "load_library"]

hid_t = ctypes.c_int64
herr_t = ctypes.c_int
hsize_t = ctypes.c_uint64
H5F_ACC_RDONLY, H5F_ACC_RDWR, H5F_ACC_TRUNC = 0, 1, 2
H5P_DEFAULT, H5S_ALL, H5S_SELECT_SET = 0, 0, 0
H5S_UNLIMITED = ctypes.c_uint64(-1).value
H5_INDEX_NAME, H5_ITER_INC = 0, 0

_lib = None


def load_library():
    """libhdf5: $MST_LIBHDF5, the loader's search path, or the image's /opt/conda copy."""
    global _lib
    if _lib is not None:
        return _lib
    cands = [os.environ.get("MST_LIBHDF5"), ctypes.util.find_library("hdf5"),
             "/opt/conda/lib/libhdf5.so.103", "/opt/conda/lib/libhdf5.so"]
    err = None
    for c in cands:
        if not c:
            continue
        try:
            lib = ctypes.CDLL(c)
            break
        except OSError as e:
            err = e
    else:
        raise ImportError("libhdf5 not found (set MST_LIBHDF5): %s" % err)
    sig = {
        "H5open": (herr_t, []),
        "H5Fopen": (hid_t, [ctypes.c_char_p, ctypes.c_uint, hid_t]),
        "H5Fcreate": (hid_t, [ctypes.c_char_p, ctypes.c_uint, hid_t, hid_t]),
        "H5Fclose": (herr_t, [hid_t]),
        "H5Dopen2": (hid_t, [hid_t, ctypes.c_char_p, hid_t]),
        "H5Dcreate2": (hid_t, [hid_t, ctypes.c_char_p, hid_t, hid_t, hid_t, hid_t, hid_t]),
        "H5Dget_space": (hid_t, [hid_t]),
        "H5Dread": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p]),
        "H5Dwrite": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p]),
        "H5Dset_extent": (herr_t, [hid_t, ctypes.POINTER(hsize_t)]),
        "H5Dclose": (herr_t, [hid_t]),
        "H5Screate_simple": (hid_t, [ctypes.c_int, ctypes.POINTER(hsize_t), ctypes.POINTER(hsize_t)]),
        "H5Sget_simple_extent_ndims": (ctypes.c_int, [hid_t]),
        "H5Sget_simple_extent_dims": (ctypes.c_int, [hid_t, ctypes.POINTER(hsize_t),
                                                     ctypes.POINTER(hsize_t)]),
        "H5Sselect_hyperslab": (herr_t, [hid_t, ctypes.c_int, ctypes.POINTER(hsize_t),
                                         ctypes.POINTER(hsize_t), ctypes.POINTER(hsize_t),
                                         ctypes.POINTER(hsize_t)]),
        "H5Sclose": (herr_t, [hid_t]),
        "H5Pcreate": (hid_t, [hid_t]),
        "H5Pset_chunk": (herr_t, [hid_t, ctypes.c_int, ctypes.POINTER(hsize_t)]),
        "H5Pclose": (herr_t, [hid_t]),
        "H5Gget_info": (herr_t, [hid_t, ctypes.c_void_p]),
        "H5Lget_name_by_idx": (ctypes.c_ssize_t, [hid_t, ctypes.c_char_p, ctypes.c_int,
                                                  ctypes.c_int, hsize_t, ctypes.c_char_p,
                                                  ctypes.c_size_t, hid_t]),
        "H5Lexists": (ctypes.c_int, [hid_t, ctypes.c_char_p, hid_t]),
        "H5Eset_auto2": (herr_t, [hid_t, ctypes.c_void_p, ctypes.c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype, f.argtypes = res, args
    if lib.H5open() < 0:
        raise ImportError("H5open failed")
    lib.H5Eset_auto2(0, None, None)  # errors come back as return codes, not stderr dumps
    lib.native_double = hid_t.in_dll(lib, "H5T_NATIVE_DOUBLE_g").value
    lib.ieee_f64le = hid_t.in_dll(lib, "H5T_IEEE_F64LE_g").value
    lib.dcpl_class = hid_t.in_dll(lib, "H5P_CLS_DATASET_CREATE_ID_g").value
    _lib = lib
    return lib


def _ck(v, what):
    if v < 0:
        raise OSError("HDF5 %s failed" % what)
    return v


def _dims(seq):
    return (hsize_t * len(seq))(*[int(s) for s in seq])


def _guess_chunk(shape, itemsize):
    """h5py's chunks=True heuristic (h5py/_hl/filters.py guess_chunk): start from the shape
    (unlimited axes as 1024), halve axes in turn until the chunk is within the target size
    derived from the dataset size (8 KiB .. 1 MiB, doubling per 10x of the total)."""
    CHUNK_BASE, CHUNK_MIN, CHUNK_MAX = 16 * 1024, 8 * 1024, 1024 * 1024
    shape = tuple((x if x != 0 else 1024) for x in shape)
    chunks = np.array(shape, dtype="=f8")
    dset_size = np.prod(chunks) * itemsize
    target = CHUNK_BASE * (2 ** np.log10(dset_size / (1024. * 1024)))
    target = min(max(target, CHUNK_MIN), CHUNK_MAX)
    idx = 0
    while True:
        chunk_bytes = np.prod(chunks) * itemsize
        if (chunk_bytes < target or abs(chunk_bytes - target) / target < 0.5) and \
                chunk_bytes < CHUNK_MAX:
            break
        if np.prod(chunks) == 1:
            break
        chunks[idx % len(shape)] = np.ceil(chunks[idx % len(shape)] / 2.0)
        idx += 1
    return tuple(int(x) for x in chunks)


class Dataset:
    def __init__(self, f, name):
        self._f, self.name = f, name

    def _open(self):
        lib = self._f._lib
        return _ck(lib.H5Dopen2(self._f._id, self.name.encode(), H5P_DEFAULT), "H5Dopen2 " + self.name)

    @property
    def shape(self):
        lib = self._f._lib
        d = self._open()
        try:
            s = _ck(lib.H5Dget_space(d), "H5Dget_space")
            n = lib.H5Sget_simple_extent_ndims(s)
            dims = (hsize_t * n)()
            lib.H5Sget_simple_extent_dims(s, dims, None)
            lib.H5Sclose(s)
            return tuple(int(x) for x in dims)
        finally:
            lib.H5Dclose(d)

    def __len__(self):
        return self.shape[0]

    def _rows(self, key, n0):
        if isinstance(key, slice):
            a, b, st = key.indices(n0)
            if st != 1:
                raise ValueError("only unit-stride row slices are supported")
            return a, max(a, b)
        if isinstance(key, (int, np.integer)):
            k = int(key) + (n0 if key < 0 else 0)
            if not 0 <= k < n0:
                raise IndexError(key)
            return k, k + 1
        raise TypeError("row index must be an int or a slice")

    def __getitem__(self, key):
        lib = self._f._lib
        shape = self.shape
        a, b = self._rows(key, shape[0])
        out = np.empty((b - a,) + shape[1:], dtype=np.float64)
        if b > a:
            self._io(a, b, out, write=False)
        return out[0] if isinstance(key, (int, np.integer)) else out

    def __setitem__(self, key, value):
        shape = self.shape
        a, b = self._rows(key, shape[0])
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(value, np.float64),
                                                 (b - a,) + shape[1:]))
        if b > a:
            self._io(a, b, v, write=True)

    def _io(self, a, b, buf, write):
        lib = self._f._lib
        shape = self.shape
        d = self._open()
        fs = _ck(lib.H5Dget_space(d), "H5Dget_space")
        try:
            start = _dims((a,) + (0,) * (len(shape) - 1))
            count = _dims((b - a,) + shape[1:])
            _ck(lib.H5Sselect_hyperslab(fs, H5S_SELECT_SET, start, None, count, None), "hyperslab")
            ms = _ck(lib.H5Screate_simple(len(shape), count, None), "H5Screate_simple")
            fn = lib.H5Dwrite if write else lib.H5Dread
            _ck(fn(d, lib.native_double, ms, fs, H5P_DEFAULT, buf.ctypes.data_as(ctypes.c_void_p)),
                "H5Dwrite" if write else "H5Dread")
            lib.H5Sclose(ms)
        finally:
            lib.H5Sclose(fs)
            lib.H5Dclose(d)

    def resize(self, size, axis=0):
        if axis != 0:
            raise ValueError("only axis 0 is resizable in this schema")
        lib = self._f._lib
        d = self._open()
        try:
            _ck(lib.H5Dset_extent(d, _dims((size,) + self.shape[1:])), "H5Dset_extent")
        finally:
            lib.H5Dclose(d)


class File:
    """h5py.File(path, mode) for the reference's datasets; mode 'r', 'r+', 'w'."""

    def __init__(self, path, mode="r"):
        self._lib = lib = load_library()
        p = os.fsencode(path)
        if mode == "r":
            self._id = lib.H5Fopen(p, H5F_ACC_RDONLY, H5P_DEFAULT)
        elif mode in ("r+", "a"):
            self._id = lib.H5Fopen(p, H5F_ACC_RDWR, H5P_DEFAULT)
        elif mode == "w":
            self._id = lib.H5Fcreate(p, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT)
        else:
            raise ValueError("mode must be 'r', 'r+' or 'w'")
        _ck(self._id, "open %s" % path)

    def keys(self):
        lib = self._lib
        info = (ctypes.c_byte * 64)()  # H5G_info_t: storage_type (int), nlinks (hsize_t), ...
        _ck(lib.H5Gget_info(self._id, info), "H5Gget_info")
        nlinks = ctypes.cast(ctypes.addressof(info) + 8, ctypes.POINTER(hsize_t))[0]
        names = []
        for i in range(nlinks):
            n = lib.H5Lget_name_by_idx(self._id, b".", H5_INDEX_NAME, H5_ITER_INC, i, None, 0,
                                       H5P_DEFAULT)
            buf = ctypes.create_string_buffer(n + 1)
            lib.H5Lget_name_by_idx(self._id, b".", H5_INDEX_NAME, H5_ITER_INC, i, buf, n + 1,
                                   H5P_DEFAULT)
            names.append(buf.value.decode())
        return names

    def __contains__(self, name):
        return self._lib.H5Lexists(self._id, name.encode(), H5P_DEFAULT) > 0

    def __getitem__(self, name):
        if name not in self:
            raise KeyError(name)
        return Dataset(self, name)

    def create_dataset(self, name, data, dtype="float64", maxshape=None, chunks=True):
        if np.dtype(dtype) != np.float64:
            raise ValueError("the reference schema is float64")
        lib = self._lib
        data = np.ascontiguousarray(data, dtype=np.float64)
        shape = data.shape
        maxshape = maxshape or shape
        maxd = _dims([H5S_UNLIMITED if m is None else m for m in maxshape])
        s = _ck(lib.H5Screate_simple(len(shape), _dims(shape), maxd), "H5Screate_simple")
        dcpl = _ck(lib.H5Pcreate(lib.dcpl_class), "H5Pcreate")
        if chunks:
            ch = _guess_chunk(shape, 8) if chunks is True else chunks
            ch = tuple(max(1, min(c, m)) if m is not None else c for c, m in zip(ch, maxshape))
            _ck(lib.H5Pset_chunk(dcpl, len(ch), _dims(ch)), "H5Pset_chunk")
        d = _ck(lib.H5Dcreate2(self._id, name.encode(), lib.ieee_f64le, s, H5P_DEFAULT, dcpl,
                               H5P_DEFAULT), "H5Dcreate2 " + name)
        if data.size:
            _ck(lib.H5Dwrite(d, lib.native_double, H5S_ALL, H5S_ALL, H5P_DEFAULT,
                             data.ctypes.data_as(ctypes.c_void_p)), "H5Dwrite")
        lib.H5Dclose(d)
        lib.H5Pclose(dcpl)
        lib.H5Sclose(s)
        return Dataset(self, name)

    def close(self):
        if getattr(self, "_id", -1) >= 0:
            self._lib.H5Fclose(self._id)
            self._id = -1

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
