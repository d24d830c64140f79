/* Per-gate fast path of the Python binding (CPython C API, no ctypes).
 *
 * A Register's one- and two-qubit gate methods (h, rx, cnot, ...) are called
 * once per gate -- 1.5-1.8 us each through ctypes (argument conversion of the
 * by-value Qureg struct, the wrapper's frames), about ten times what the
 * library itself spends queueing the gate (0.16 us).  At 26 qubits a 10-layer
 * window issues 390 gates before the GPU starts: the binding's overhead was
 * ~15 % of the window.  This module binds the same exported C functions
 * (resolved by ctypes, passed here as addresses) to a per-register object
 * whose methods call them directly: same API functions, same validation and
 * error handler (an error sets `errflag`; the method then calls the Python
 * binding's check(), which raises QuESTError), the same QASM recording.  As
 * ctypes does, the call runs without the GIL (a gate can start a flush that
 * waits for the GPU); the error handler is a ctypes callback, which takes the
 * GIL itself.
 *
 * QuEST.h's Qureg holds only ints and pointers, so one layout serves every
 * precision; the angle argument's C type follows the loaded library's
 * QuEST_PREC (float / double / long double).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <limits.h>
#include <string.h>

#include "QuEST.h"

enum {
    F_H, F_X, F_Y, F_Z, F_S, F_T,          /* (Qureg, int) */
    F_RX, F_RY, F_RZ, F_PHASE,             /* (Qureg, int, qreal) */
    F_CNOT, F_CY, F_CZ,                    /* (Qureg, int, int) */
    F_CRX, F_CRY, F_CRZ, F_CPHASE,         /* (Qureg, int, int, qreal) */
    F_COUNT
};

typedef void (*Fn1)(Qureg, int);
typedef void (*Fn2)(Qureg, int, int);
typedef void (*Fn1f)(Qureg, int, float);
typedef void (*Fn1d)(Qureg, int, double);
typedef void (*Fn1l)(Qureg, int, long double);
typedef void (*Fn2f)(Qureg, int, int, float);
typedef void (*Fn2d)(Qureg, int, int, double);
typedef void (*Fn2l)(Qureg, int, int, long double);

static void* g_fn[F_COUNT];
static int g_prec = 0;               /* 0: not initialised */
static volatile int* g_errflag = NULL;
static PyObject* g_check = NULL;     /* the binding's check(): raises QuESTError */

typedef struct {
    PyObject_HEAD
    Qureg q;
    int alive;
} Gates;

/* An int argument as the C API's int: values outside int become -1, which
 * every target / control validation rejects (ctypes would have wrapped). */
static int argInt(PyObject* o, int* out) {
    int overflow = 0;
    const long v = PyLong_AsLongAndOverflow(o, &overflow);
    if (v == -1 && PyErr_Occurred()) return -1;
    *out = (overflow || v < INT_MIN || v > INT_MAX) ? -1 : (int)v;
    return 0;
}

static int ready(Gates* g, Py_ssize_t nargs, Py_ssize_t want, const char* name) {
    if (!g->alive) {
        PyErr_Format(PyExc_RuntimeError, "%s: register is closed", name);
        return 0;
    }
    if (nargs != want) {
        PyErr_Format(PyExc_TypeError, "%s() takes %zd arguments (%zd given)", name, want, nargs);
        return 0;
    }
    return 1;
}

/* after every call: an error the handler recorded becomes the exception */
static PyObject* done(void) {
    if (*g_errflag) {
        PyObject* r = PyObject_CallNoArgs(g_check);
        if (!r) return NULL;
        Py_DECREF(r);
    }
    Py_RETURN_NONE;
}

static PyObject* call1(Gates* g, PyObject* const* a, Py_ssize_t n, int f, const char* name) {
    int t;
    if (!ready(g, n, 1, name) || argInt(a[0], &t)) return NULL;
    Py_BEGIN_ALLOW_THREADS
    ((Fn1)g_fn[f])(g->q, t);
    Py_END_ALLOW_THREADS
    return done();
}

static PyObject* call2(Gates* g, PyObject* const* a, Py_ssize_t n, int f, const char* name) {
    int c, t;
    if (!ready(g, n, 2, name) || argInt(a[0], &c) || argInt(a[1], &t)) return NULL;
    Py_BEGIN_ALLOW_THREADS
    ((Fn2)g_fn[f])(g->q, c, t);
    Py_END_ALLOW_THREADS
    return done();
}

static PyObject* call1a(Gates* g, PyObject* const* a, Py_ssize_t n, int f, const char* name) {
    int t;
    if (!ready(g, n, 2, name) || argInt(a[0], &t)) return NULL;
    const double x = PyFloat_AsDouble(a[1]);
    if (x == -1.0 && PyErr_Occurred()) return NULL;
    Py_BEGIN_ALLOW_THREADS
    if (g_prec == 1)
        ((Fn1f)g_fn[f])(g->q, t, (float)x);
    else if (g_prec == 4)
        ((Fn1l)g_fn[f])(g->q, t, (long double)x);
    else
        ((Fn1d)g_fn[f])(g->q, t, x);
    Py_END_ALLOW_THREADS
    return done();
}

static PyObject* call2a(Gates* g, PyObject* const* a, Py_ssize_t n, int f, const char* name) {
    int c, t;
    if (!ready(g, n, 3, name) || argInt(a[0], &c) || argInt(a[1], &t)) return NULL;
    const double x = PyFloat_AsDouble(a[2]);
    if (x == -1.0 && PyErr_Occurred()) return NULL;
    Py_BEGIN_ALLOW_THREADS
    if (g_prec == 1)
        ((Fn2f)g_fn[f])(g->q, c, t, (float)x);
    else if (g_prec == 4)
        ((Fn2l)g_fn[f])(g->q, c, t, (long double)x);
    else
        ((Fn2d)g_fn[f])(g->q, c, t, x);
    Py_END_ALLOW_THREADS
    return done();
}

#define M1(py, F)                                                                      \
    static PyObject* m_##py(PyObject* s, PyObject* const* a, Py_ssize_t n) {           \
        return call1((Gates*)s, a, n, F, #py);                                         \
    }
#define M2(py, F)                                                                      \
    static PyObject* m_##py(PyObject* s, PyObject* const* a, Py_ssize_t n) {           \
        return call2((Gates*)s, a, n, F, #py);                                         \
    }
#define M1A(py, F)                                                                     \
    static PyObject* m_##py(PyObject* s, PyObject* const* a, Py_ssize_t n) {           \
        return call1a((Gates*)s, a, n, F, #py);                                        \
    }
#define M2A(py, F)                                                                     \
    static PyObject* m_##py(PyObject* s, PyObject* const* a, Py_ssize_t n) {           \
        return call2a((Gates*)s, a, n, F, #py);                                        \
    }

M1(h, F_H)
M1(x, F_X)
M1(y, F_Y)
M1(z, F_Z)
M1(s, F_S)
M1(t, F_T)
M1A(rx, F_RX)
M1A(ry, F_RY)
M1A(rz, F_RZ)
M1A(phase, F_PHASE)
M2(cnot, F_CNOT)
M2(cy, F_CY)
M2(cz, F_CZ)
M2A(crx, F_CRX)
M2A(cry, F_CRY)
M2A(crz, F_CRZ)
M2A(cphase, F_CPHASE)

static PyObject* m_close(PyObject* s, PyObject* unused) {
    (void)unused;
    ((Gates*)s)->alive = 0;
    Py_RETURN_NONE;
}

#define ENTRY(py) {#py, (PyCFunction)(void (*)(void))m_##py, METH_FASTCALL, NULL}
static PyMethodDef gates_methods[] = {
    ENTRY(h),   ENTRY(x),    ENTRY(y),     ENTRY(z),   ENTRY(s),   ENTRY(t),
    ENTRY(rx),  ENTRY(ry),   ENTRY(rz),    ENTRY(phase),
    ENTRY(cnot), ENTRY(cy),  ENTRY(cz),
    ENTRY(crx), ENTRY(cry),  ENTRY(crz),   ENTRY(cphase),
    {"close", m_close, METH_NOARGS, "Stop calling into the register (destroyQureg follows)."},
    {NULL, NULL, 0, NULL}};

static PyTypeObject GatesType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "quest_amd.ops._gatecall.Gates",
    .tp_basicsize = sizeof(Gates),
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "Gate methods of one register, calling the C API directly.",
    .tp_methods = gates_methods,
};

/* configure(addresses, prec, errflag_address, check) -- addresses in the
 * order of the F_* enum */
static PyObject* configure(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *addrs, *check;
    int prec;
    unsigned long long errAddr;
    if (!PyArg_ParseTuple(args, "OiKO", &addrs, &prec, &errAddr, &check)) return NULL;
    if (prec != 1 && prec != 2 && prec != 4) return PyErr_Format(PyExc_ValueError, "precision %d", prec);
    PyObject* seq = PySequence_Fast(addrs, "addresses must be a sequence");
    if (!seq) return NULL;
    if (PySequence_Fast_GET_SIZE(seq) != F_COUNT) {
        Py_DECREF(seq);
        return PyErr_Format(PyExc_ValueError, "expected %d addresses", F_COUNT);
    }
    void* fns[F_COUNT];
    for (int i = 0; i < F_COUNT; i++) {
        const unsigned long long v = PyLong_AsUnsignedLongLong(PySequence_Fast_GET_ITEM(seq, i));
        if (PyErr_Occurred()) {
            Py_DECREF(seq);
            return NULL;
        }
        if (!v) {
            Py_DECREF(seq);
            return PyErr_Format(PyExc_ValueError, "null address %d", i);
        }
        fns[i] = (void*)(uintptr_t)v;
    }
    Py_DECREF(seq);
    if (!errAddr || !PyCallable_Check(check)) return PyErr_Format(PyExc_ValueError, "error flag / check");
    memcpy(g_fn, fns, sizeof fns);
    g_prec = prec;
    g_errflag = (volatile int*)(uintptr_t)errAddr;
    Py_INCREF(check);
    Py_XSETREF(g_check, check);
    Py_RETURN_NONE;
}

/* bind(qureg_address, qureg_size) -> Gates: a copy of the ctypes Qureg */
static PyObject* bind(PyObject* self, PyObject* args) {
    (void)self;
    unsigned long long addr;
    Py_ssize_t size;
    if (!PyArg_ParseTuple(args, "Kn", &addr, &size)) return NULL;
    if (!g_prec) return PyErr_Format(PyExc_RuntimeError, "configure() first");
    if (size != (Py_ssize_t)sizeof(Qureg))
        return PyErr_Format(PyExc_ValueError, "Qureg is %zd bytes here, %zd in the binding", (Py_ssize_t)sizeof(Qureg),
                            size);
    Gates* g = PyObject_New(Gates, &GatesType);
    if (!g) return NULL;
    memcpy(&g->q, (const void*)(uintptr_t)addr, sizeof(Qureg));
    g->alive = 1;
    return (PyObject*)g;
}

static PyObject* qureg_size(PyObject* self, PyObject* unused) {
    (void)self;
    (void)unused;
    return PyLong_FromSsize_t((Py_ssize_t)sizeof(Qureg));
}

static PyMethodDef module_methods[] = {
    {"configure", configure, METH_VARARGS, "Function addresses, QuEST_PREC, error flag address, check callable."},
    {"bind", bind, METH_VARARGS, "Gates object for a Qureg (address, size)."},
    {"qureg_size", qureg_size, METH_NOARGS, "sizeof(Qureg) in this build."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef moduledef = {PyModuleDef_HEAD_INIT, "_gatecall",
                                       "Per-gate fast path of the quest_amd binding.", -1, module_methods};

PyMODINIT_FUNC PyInit__gatecall(void) {
    if (PyType_Ready(&GatesType) < 0) return NULL;
    PyObject* m = PyModule_Create(&moduledef);
    if (!m) return NULL;
    /* the enum order, for the Python side */
    PyObject* names = Py_BuildValue("(sssssssssssssssss)", "hadamard", "pauliX", "pauliY", "pauliZ", "sGate", "tGate",
                                    "rotateX", "rotateY", "rotateZ", "phaseShift", "controlledNot",
                                    "controlledPauliY", "controlledPhaseFlip", "controlledRotateX",
                                    "controlledRotateY", "controlledRotateZ", "controlledPhaseShift");
    if (!names || PyModule_AddObject(m, "FUNCTIONS", names) < 0) {
        Py_XDECREF(names);
        Py_DECREF(m);
        return NULL;
    }
    return m;
}
