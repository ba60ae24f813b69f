// Native ingestion of (key, vector) records — the reference's RDD element
// form (R:dbscan/dbscan.py:104-109: ``data`` is an RDD of (key, k-dim
// vector)) — into one contiguous (n, d) coordinate buffer and an int64 key
// buffer, for the H2D copy of as_points().  A CPython extension (no numpy C
// API: the caller passes preallocated buffers through the buffer protocol).
//
// unzip(records, X, K, d, f64) -> status
//   records: list / tuple of 2-sequences (key, vector); vector: any buffer of
//            d float32 / float64 values (numpy rows) or a sequence of numbers
//   X:       writable C-contiguous buffer of n*d float32 (f64 = 0) or float64
//   K:       writable C-contiguous buffer of n int64
//   status:  bit 0 set = every key was an int that fits int64 (K holds them);
//            2 = a vector was not float32 while X is float32 (retry with
//            f64 = 1: the caller keeps float32 only when every vector is)
// Raises TypeError / ValueError on malformed records.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstring>

namespace {

struct Buf {
    Py_buffer b{};
    bool ok = false;
    Buf(PyObject* o, int flags) { ok = PyObject_GetBuffer(o, &b, flags) == 0; }
    ~Buf() {
        if (ok) PyBuffer_Release(&b);
    }
};

// 'f' / 'd' (optionally with a byte-order prefix the host shares)
char fmt_code(const char* f) {
    if (!f) return 'B';
    if (*f == '<' || *f == '=' || *f == '@') ++f;
    return *f;
}

PyObject* unzip(PyObject*, PyObject* args) {
    PyObject *recs, *xo, *ko;
    int d = 0, f64 = 0;
    if (!PyArg_ParseTuple(args, "OOOii", &recs, &xo, &ko, &d, &f64)) return nullptr;
    if (d < 1) {
        PyErr_SetString(PyExc_ValueError, "d must be >= 1");
        return nullptr;
    }
    PyObject* fast = PySequence_Fast(recs, "records must be a sequence of (key, vector)");
    if (!fast) return nullptr;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
    PyObject** items = PySequence_Fast_ITEMS(fast);
    Buf xb(xo, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS), kb(ko, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS);
    if (!xb.ok || !kb.ok) {
        Py_DECREF(fast);
        return nullptr;
    }
    const Py_ssize_t isz = f64 ? 8 : 4;
    if (xb.b.len < n * d * isz || kb.b.len < n * 8) {
        Py_DECREF(fast);
        PyErr_SetString(PyExc_ValueError, "output buffers too small");
        return nullptr;
    }
    char* xp = (char*)xb.b.buf;
    long long* kp = (long long*)kb.b.buf;
    bool keys_int = true;
    long status = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* r = items[i];
        PyObject *key, *vec;
        if (PyTuple_Check(r) && PyTuple_GET_SIZE(r) == 2) {
            key = PyTuple_GET_ITEM(r, 0);
            vec = PyTuple_GET_ITEM(r, 1);
        } else if (PyList_Check(r) && PyList_GET_SIZE(r) == 2) {
            key = PyList_GET_ITEM(r, 0);
            vec = PyList_GET_ITEM(r, 1);
        } else {
            Py_DECREF(fast);
            PyErr_Format(PyExc_TypeError, "record %zd is not a (key, vector) pair", i);
            return nullptr;
        }
        if (keys_int) {
            if (PyLong_Check(key) && !PyBool_Check(key)) {
                int of = 0;
                const long long v = PyLong_AsLongLongAndOverflow(key, &of);
                if (of || (v == -1 && PyErr_Occurred())) {
                    PyErr_Clear();
                    keys_int = false;
                } else {
                    kp[i] = v;
                }
            } else {
                keys_int = false;
            }
        }
        char* dst = xp + i * d * isz;
        bool done = false;
        if (PyObject_CheckBuffer(vec)) {
            // strided 1-D views (a column slice of a matrix) are accepted too
            Buf vb(vec, PyBUF_FORMAT | PyBUF_STRIDES);
            if (vb.ok && vb.b.ndim == 1) {
                const char c = fmt_code(vb.b.format);
                const Py_ssize_t cnt = vb.b.shape[0], st = vb.b.strides[0];
                if (cnt != d) {
                    Py_DECREF(fast);
                    PyErr_Format(PyExc_ValueError, "record %zd: vector of %zd values, expected %d",
                                 i, cnt, d);
                    return nullptr;
                }
                const char* s = (const char*)vb.b.buf;
                if (c == 'f' && vb.b.itemsize == 4) {
                    if (f64)
                        for (int j = 0; j < d; ++j)
                            ((double*)dst)[j] = (double)*(const float*)(s + j * st);
                    else if (st == 4)
                        std::memcpy(dst, s, 4 * (size_t)d);
                    else
                        for (int j = 0; j < d; ++j) ((float*)dst)[j] = *(const float*)(s + j * st);
                    done = true;
                } else if (c == 'd' && vb.b.itemsize == 8) {
                    if (!f64) {   // float64 data: the set is float64
                        Py_DECREF(fast);
                        return PyLong_FromLong(2);
                    }
                    if (st == 8)
                        std::memcpy(dst, s, 8 * (size_t)d);
                    else
                        for (int j = 0; j < d; ++j) ((double*)dst)[j] = *(const double*)(s + j * st);
                    done = true;
                }
            } else if (!vb.ok) {
                PyErr_Clear();
            }
        }
        if (!done) {   // a sequence of numbers (or a buffer of another type)
            if (!f64) {
                Py_DECREF(fast);
                return PyLong_FromLong(2);
            }
            PyObject* vf = PySequence_Fast(vec, "vector must be a sequence of numbers");
            if (!vf) {
                Py_DECREF(fast);
                return nullptr;
            }
            if (PySequence_Fast_GET_SIZE(vf) != d) {
                Py_DECREF(vf);
                Py_DECREF(fast);
                PyErr_Format(PyExc_ValueError, "record %zd: vector of the wrong length", i);
                return nullptr;
            }
            PyObject** vi = PySequence_Fast_ITEMS(vf);
            for (int j = 0; j < d; ++j) {
                const double v = PyFloat_AsDouble(vi[j]);
                if (v == -1.0 && PyErr_Occurred()) {
                    Py_DECREF(vf);
                    Py_DECREF(fast);
                    return nullptr;
                }
                ((double*)dst)[j] = v;
            }
            Py_DECREF(vf);
        }
    }
    Py_DECREF(fast);
    status = keys_int ? 1 : 0;
    return PyLong_FromLong(status);
}

PyMethodDef methods[] = {
    {"unzip", unzip, METH_VARARGS, "unzip(records, X, K, d, f64) -> status"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_ingest",
                      "Native (key, vector) record ingestion (pypardis_amd)", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__ingest(void) { return PyModule_Create(&module); }
