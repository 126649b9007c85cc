/* One single-game tick for astro_amd.core.step, packing and unpacking in C.
 *
 * core.step(state, control, config) (reference: astro/core.py:215-303) runs
 * one game's tick as one astro_game_step call on a host-mapped arena
 * (include/astro_step.h).  The Python shim around that call -- the State's
 * seven arrays packed into the tick record's input, the reference's float64
 * bookkeeping of reload and t (core.py:257,263,267), the next State built
 * from the packed output -- was ~8 us of a ~23 us tick.  This module does the
 * same in C over the numpy buffers: identical values, dtypes and shapes
 * (float32 planets for a lone planet, float32 bullets at a game's first
 * tick, an int64 reward on a collision), and Python's own arithmetic for
 * reload and t (PyNumber_*), so their types follow the caller's.  Anything
 * it does not handle (non-contiguous or non-float arrays, wrong shapes)
 * returns NotImplemented and the Python path runs instead.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>

#include "astro_step.h"

typedef int (*game_step_fn)(AstroGameTick *);

/* n doubles of a C-contiguous float32/float64 array into dst; -1 if the
 * array is not one the fast path takes */
static int pack(PyObject *o, Py_ssize_t n, double *dst, int *is_f32) {
    if (!PyArray_Check(o)) return -1;
    PyArrayObject *a = (PyArrayObject *)o;
    if (PyArray_SIZE(a) != n || !PyArray_IS_C_CONTIGUOUS(a)) return -1;
    const int t = PyArray_TYPE(a);
    if (t == NPY_FLOAT64) {
        memcpy(dst, PyArray_DATA(a), (size_t)n * sizeof(double));
        if (is_f32) *is_f32 = 0;
    } else if (t == NPY_FLOAT32) {
        const float *s = (const float *)PyArray_DATA(a);
        for (Py_ssize_t k = 0; k < n; ++k) dst[k] = (double)s[k];
        if (is_f32) *is_f32 = 1;
    } else {
        return -1;
    }
    return 0;
}

static Py_ssize_t rows_of(PyObject *o) {
    if (!PyArray_Check(o) || PyArray_NDIM((PyArrayObject *)o) < 1) return -1;
    return PyArray_DIM((PyArrayObject *)o, 0);
}

/* a new [rows, cols] (cols 0: [rows]) array of src, float64 or float32 */
static PyObject *unpack(const double *src, npy_intp rows, npy_intp cols, int f32) {
    npy_intp dims[2] = {rows, cols};
    PyObject *o = PyArray_SimpleNew(cols ? 2 : 1, dims, f32 ? NPY_FLOAT32 : NPY_FLOAT64);
    if (!o) return NULL;
    const npy_intp n = rows * (cols ? cols : 1);
    if (f32) {
        float *d = (float *)PyArray_DATA((PyArrayObject *)o);
        for (npy_intp k = 0; k < n; ++k) d[k] = (float)src[k];
    } else {
        memcpy(PyArray_DATA((PyArrayObject *)o), src, (size_t)n * sizeof(double));
    }
    return o;
}

static PyObject *bodies(PyObject *Bodies, PyObject *x, PyObject *dx, PyObject *b) {
    if (!x || !dx || !b) {
        Py_XDECREF(x);
        Py_XDECREF(dx);
        Py_XDECREF(b);
        return NULL;
    }
    PyObject *r = PyObject_CallFunctionObjArgs(Bodies, x, dx, b, NULL);
    Py_DECREF(x);
    Py_DECREF(dx);
    Py_DECREF(b);
    return r;
}

/* step(tick_addr, fn_addr, state, c0, c1, dt, reload_time, max_time, State, Bodies)
 *   -> (State or None, reward) | int rc (< 0: astro_game_step failed) | NotImplemented */
static PyObject *gs_step(PyObject *self, PyObject *args) {
    unsigned long long tick_addr, fn_addr;
    PyObject *state, *dt, *reload_time, *max_time, *State, *Bodies;
    int c0, c1;
    if (!PyArg_ParseTuple(args, "KKOiiOOOOO", &tick_addr, &fn_addr, &state, &c0, &c1, &dt, &reload_time, &max_time,
                          &State, &Bodies))
        return NULL;
    AstroGameTick *t = (AstroGameTick *)(uintptr_t)tick_addr;
    game_step_fn fn = (game_step_fn)(uintptr_t)fn_addr;
    if (!PyTuple_Check(state) || PyTuple_GET_SIZE(state) != 5) Py_RETURN_NOTIMPLEMENTED;
    PyObject *ships = PyTuple_GET_ITEM(state, 0), *planets = PyTuple_GET_ITEM(state, 1),
             *bullets = PyTuple_GET_ITEM(state, 2), *reload = PyTuple_GET_ITEM(state, 3),
             *tt = PyTuple_GET_ITEM(state, 4);
    if (!PyTuple_Check(ships) || PyTuple_GET_SIZE(ships) != 3 || !PyTuple_Check(planets) ||
        PyTuple_GET_SIZE(planets) != 3 || !PyTuple_Check(bullets) || PyTuple_GET_SIZE(bullets) != 3)
        Py_RETURN_NOTIMPLEMENTED;
    const int S = t->params.nships;
    const Py_ssize_t npl = rows_of(PyTuple_GET_ITEM(planets, 0)), nb = rows_of(PyTuple_GET_ITEM(bullets, 0));
    if (npl < 1 || npl > t->params.p_pad || nb < 0 || nb > t->params.b_cap) Py_RETURN_NOTIMPLEMENTED;
    /* the input, packed as the shim's: ships x, dx, b, planets x, dx, bullets x, dx */
    double *in = (double *)t->in;
    int fresh = 0, f;
    if (pack(PyTuple_GET_ITEM(ships, 0), 2 * S, in, &fresh) || pack(PyTuple_GET_ITEM(ships, 1), 2 * S, in + 2 * S, &f) ||
        pack(PyTuple_GET_ITEM(ships, 2), S, in + 4 * S, &f) ||
        pack(PyTuple_GET_ITEM(planets, 0), 2 * npl, in + 5 * S, &f) ||
        pack(PyTuple_GET_ITEM(planets, 1), 2 * npl, in + 5 * S + 2 * npl, &f) ||
        pack(PyTuple_GET_ITEM(bullets, 0), 2 * nb, in + 5 * S + 4 * npl, &f) ||
        pack(PyTuple_GET_ITEM(bullets, 1), 2 * nb, in + 5 * S + 4 * npl + 2 * nb, &f))
        Py_RETURN_NOTIMPLEMENTED;
    /* the reference's float64 bookkeeping for THIS call (core.py:257,263,267) */
    PyObject *r_next = PyNumber_Add(reload, dt);
    if (!r_next) return NULL;
    PyObject *t_next = PyNumber_Add(tt, dt);
    if (!t_next) {
        Py_DECREF(r_next);
        return NULL;
    }
    const int fire = PyObject_RichCompareBool(reload_time, r_next, Py_LE);
    const int timeout = PyObject_RichCompareBool(max_time, t_next, Py_LE);
    if (fire < 0 || timeout < 0) {
        Py_DECREF(r_next);
        Py_DECREF(t_next);
        return NULL;
    }
    t->nplanets = (int32_t)npl;
    t->nbullets = (int32_t)nb;
    t->control0 = c0;
    t->control1 = c1;
    t->first_step = fresh;
    t->fire_now = fire;
    t->timeout_now = timeout;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = fn(t);
    Py_END_ALLOW_THREADS
    if (rc != 0) {
        Py_DECREF(r_next);
        Py_DECREF(t_next);
        return PyLong_FromLong(rc);
    }
    if (t->done_out) {   /* (None, reward): int64 on a collision, float32 on the timeout */
        Py_DECREF(r_next);
        Py_DECREF(t_next);
        npy_intp dims[1] = {S};
        PyObject *rw = PyArray_SimpleNew(1, dims, t->done_out == 1 ? NPY_INT64 : NPY_FLOAT32);
        if (!rw) return NULL;
        for (int s = 0; s < S; ++s) {
            if (t->done_out == 1)
                ((npy_int64 *)PyArray_DATA((PyArrayObject *)rw))[s] = (npy_int64)t->reward_out[s];
            else
                ((float *)PyArray_DATA((PyArrayObject *)rw))[s] = t->reward_out[s];
        }
        return Py_BuildValue("(ON)", Py_None, rw);
    }
    if (fire) {
        PyObject *r2 = PyNumber_Subtract(r_next, reload_time);
        Py_DECREF(r_next);
        if (!r2) {
            Py_DECREF(t_next);
            return NULL;
        }
        r_next = r2;
    }
    const double *o = t->out;
    const int nb2 = t->out_nbullets;
    const double *po = o + 5 * S, *bo = o + 5 * S + 4 * npl;
    PyObject *sh = bodies(Bodies, unpack(o, S, 2, 0), unpack(o + 2 * S, S, 2, 0), unpack(o + 4 * S, S, 0, 0));
    Py_INCREF(Py_None);
    Py_INCREF(Py_None);
    PyObject *pl = bodies(Bodies, unpack(po, npl, 2, npl == 1), unpack(po + 2 * npl, npl, 2, npl == 1), Py_None);
    PyObject *bu = bodies(Bodies, unpack(bo, nb2, 2, fresh), unpack(bo + 2 * nb2, nb2, 2, fresh), Py_None);
    if (!sh || !pl || !bu) {
        Py_XDECREF(sh);
        Py_XDECREF(pl);
        Py_XDECREF(bu);
        Py_DECREF(r_next);
        Py_DECREF(t_next);
        return NULL;
    }
    PyObject *ns = PyObject_CallFunctionObjArgs(State, sh, pl, bu, r_next, t_next, NULL);
    Py_DECREF(sh);
    Py_DECREF(pl);
    Py_DECREF(bu);
    Py_DECREF(r_next);
    Py_DECREF(t_next);
    if (!ns) return NULL;
    npy_intp dims[1] = {S};
    PyObject *rw = PyArray_ZEROS(1, dims, NPY_FLOAT32, 0);
    if (!rw) {
        Py_DECREF(ns);
        return NULL;
    }
    return Py_BuildValue("(NN)", ns, rw);
}

static PyMethodDef methods[] = {
    {"step", gs_step, METH_VARARGS, "one single-game tick through astro_game_step (see the module doc)"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_gamestep", NULL, -1, methods};

PyMODINIT_FUNC PyInit__gamestep(void) {
    import_array();
    return PyModule_Create(&module);
}
