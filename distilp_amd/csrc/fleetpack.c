/*
 * _fleetpack: packs lists of DeviceProfile objects into the flat device-field table of
 * halda_solve_fleets (distilp_amd/solver/fleets.py: fleet_table), in C: one pass over the devices
 * reading each profile's pydantic field dict, no per-field Python bytecode. Same values, flags and
 * exceptions as the Python packer it replaces (which restates dense_common.py:25-126 / :211-230 and
 * the reference's truthiness tests, see fleets.py), so the single-fleet halda_solve path spends
 * microseconds, not a Python loop, before the GPU call.
 *
 *   pack(fleets, Q, fq, fout, f64, b64, u8, off, heads) -> None
 *     fleets  sequence of sequences of DeviceProfile
 *     Q       the model's quantisation key; fq / fout: "b_1" in model.f_q / model.f_out
 *     f64     writable float64 buffer [10][nd] (F64_FIELDS rows), b64: float64 [6][nd] (BYTE_FIELDS rows: the
 *             integer byte counts as doubles, exact below 2^53), u8: uint8
 *     [2][nd] (os_class row, flags row), off: int64 [n_fleets + 1], heads: int64 [n_fleets]
 *   raises what fleets.fleet_table_py raises, FleetTable.check's ZeroDivisionErrors included
 */
#define PY_SSIZE_T_CLEAN
#define _GNU_SOURCE
#include <Python.h>
#include <structmember.h>
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { HEAD = 1, UMA = 2, CPU_RATE = 4, GPU = 8, GPU_RATE = 16, CUDA_OK = 32, METAL_OK = 64, METAL_AVAIL = 128 };

/* field names, interned once (a lookup hashes nothing: the key objects cache their hash) */
#define KEYS(X) X(os_type) X(is_head) X(is_unified_mem) X(scpu) X(has_metal) X(has_cuda) X(sgpu_metal) \
    X(sgpu_cuda) X(T_metal) X(T_cuda) X(d_avail_cuda) X(d_avail_metal) X(T_cpu) X(t_kvcpy_cpu) X(t_kvcpy_gpu) \
    X(t_ram2vram) X(t_vram2ram) X(t_comm) X(s_disk) X(d_avail_ram) X(c_cpu) X(c_gpu) X(d_bytes_can_swap) \
    X(d_swap_avail) X(b_1)
#define DECL(n) static PyObject *k_##n; static Py_hash_t h_##n;
KEYS(DECL)
#undef DECL

static PyObject *item_o(PyObject *d, PyObject *k) {
    PyObject *v = PyDict_GetItemWithError(d, k); /* borrowed */
    if (!v && !PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, k);
    return v;
}
#define item(d, name) item_o(d, k_##name)

static int as_f64(PyObject *v, double *out) {
    *out = PyFloat_AsDouble(v);
    return (*out == -1.0 && PyErr_Occurred()) ? -1 : 0;
}

static int as_i64(PyObject *v, int64_t *out) {
    *out = (int64_t)PyLong_AsLongLong(v);
    return (*out == -1 && PyErr_Occurred()) ? -1 : 0;
}

static int no_b1(PyObject *Q) {
    PyErr_Format(PyExc_ValueError, "Batch size 1 (key 'b_1') not found in S_by_q[%S]", Q);
    return -1;
}

/* _rate of fleets.py: (present, value) of table[Q]["b_1"]; raises when the key is missing and fq */
static int rate(PyObject *table, PyObject *Q, int fq, int *present, double *v) {
    *present = 0;
    *v = 0.0;
    if (table == Py_None || !PyDict_Check(table)) return 0;
    PyObject *row = PyDict_GetItemWithError(table, Q);
    if (!row) return PyErr_Occurred() ? -1 : 0;
    if (!PyDict_Check(row)) {
        PyErr_SetString(PyExc_TypeError, "FLOPs table row is not a dict");
        return -1;
    }
    PyObject *b1 = PyDict_GetItemWithError(row, k_b_1);
    if (!b1) return PyErr_Occurred() ? -1 : fq ? no_b1(Q) : 0;
    *present = 1;
    return as_f64(b1, v);
}

/* ---------------------------------------------------------------- fast (parallel) pass
 * Large tables are packed by several threads while the calling thread holds the GIL and waits (small
 * ones by the calling thread itself), so
 * no Python code runs and no object changes meanwhile. Each device's instance dict: on CPython < 3.11
 * _PyObject_GetDictPtr is pointer arithmetic on the object (tp_dictoffset), so the workers take it
 * themselves; from 3.11 on it may create the dict of an object whose attributes are still inline (a
 * managed dict), so there the calling thread collects every dict first, under the GIL (an object
 * without an exact str-keyed dict sends the table to the serial pass). The workers only READ:
 * the borrowed dicts, lookups by precomputed hash in str-keyed dicts
 * (_PyDict_GetItem_KnownHash: no error state, no Python code), and the values of exact float / int /
 * bool / None / str / dict objects. No reference count changes, no allocation, no exception: any
 * value outside that (a missing key, another type, an overflow, a FLOPs table without "b_1") makes the
 * worker give up, and the whole table is packed again by the serial pass below, which raises the
 * reference's exceptions in the reference's order. So the parallel pass either writes exactly what
 * the serial one would, or nothing that is kept. */
#if PY_VERSION_HEX >= 0x030B0000
#define DICTS_ON_CALLER 1 /* devs[] holds the instance dicts, collected by the calling thread */
#else
#define DICTS_ON_CALLER 0 /* devs[] holds the objects; a worker takes each one's dict (no allocation) */
#endif

/* the instance dict of entry g of devs[] (NULL: none, or not an exact str-keyed dict) */
static PyObject *dev_dict(PyObject *o) {
#if DICTS_ON_CALLER
    return o;
#else
    PyObject **dp = _PyObject_GetDictPtr(o);
    return dp && *dp && PyDict_CheckExact(*dp) ? *dp : NULL;
#endif
}

typedef struct {
    PyObject **devs; /* the devices' instance dicts (DICTS_ON_CALLER) or objects */
    Py_ssize_t lo, hi, nd;
    PyObject *Q;
    Py_hash_t hQ;
    int fq;
    double *f64;
    double *b64;
    uint8_t *cls, *flg;
    volatile int *bail;
} Job;

static PyObject *fget(PyObject *d, PyObject *k, Py_hash_t h) { return _PyDict_GetItem_KnownHash(d, k, h); }
#define FGET(d, name) fget(d, k_##name, h_##name)

static int fbool(PyObject *o, int *t) {
    if (o == Py_True) *t = 1;
    else if (o == Py_False) *t = 0;
    else return -1;
    return 0;
}
static int fdict(PyObject *o) { return o && PyDict_CheckExact(o) && _PyDict_HasOnlyStringKeys(o); }
static int ff64(PyObject *o, double *v) {
    if (!o || !PyFloat_CheckExact(o)) return -1;
    *v = PyFloat_AS_DOUBLE(o);
    return 0;
}
static int fi64(PyObject *o, int64_t *v) {
    if (!o || !PyLong_CheckExact(o)) return -1;
    int ovf = 0;
    const long long x = PyLong_AsLongLongAndOverflow(o, &ovf);
    if (ovf) return -1; /* an exact int never sets an error here */
    *v = (int64_t)x;
    return 0;
}
/* "table" truthy: a non-empty exact dict (None / empty: 0); anything else: -1 */
static int ftable(PyObject *o) {
    if (o == Py_None) return 0;
    if (!fdict(o)) return -1;
    return PyDict_GET_SIZE(o) > 0;
}
/* a load-throughput value: None / 0.0 falsy, a float truthy; anything else -1 */
static int fthru(PyObject *o) {
    if (o == Py_None) return 0;
    if (!PyFloat_CheckExact(o)) return -1;
    return PyFloat_AS_DOUBLE(o) != 0.0;
}

/* one device (its instance dict d), the serial pass's reads restricted to the plain cases; -1: give up */
static int fast_dev(const Job *J, PyObject *d, Py_ssize_t g) {
    PyObject *o;
    PyObject *os = FGET(d, os_type);
    if (!os || !PyUnicode_CheckExact(os)) return -1;
    int c = 3;
    if (PyUnicode_CompareWithASCIIString(os, "mac_no_metal") == 0) c = 1;
    else if (PyUnicode_CompareWithASCIIString(os, "mac_metal") == 0) c = 2;
    const int android = PyUnicode_CompareWithASCIIString(os, "android") == 0;
    int fl = 0, t;
    if (!(o = FGET(d, is_head)) || fbool(o, &t)) return -1;
    fl |= t ? HEAD : 0;
    if (!(o = FGET(d, is_unified_mem)) || fbool(o, &t)) return -1;
    fl |= t ? UMA : 0;
    PyObject *sc = FGET(d, scpu);
    if (!sc) return -1;
    double v = 0.0;
    const int st = ftable(sc);
    if (st < 0) return -1;
    if (st) {
        PyObject *row = _PyDict_GetItem_KnownHash(sc, J->Q, J->hQ);
        if (row && row != Py_None) {
            if (!fdict(row)) return -1;
            PyObject *b1 = FGET(row, b_1);
            if (!b1 || ff64(b1, &v)) return -1; /* b_1 missing: the serial pass decides whether it raises */
            fl |= CPU_RATE;
        }
    }
    PyObject *hm = FGET(d, has_metal), *hc = FGET(d, has_cuda);
    int has_metal, has_cuda;
    if (!hm || !hc || fbool(hm, &has_metal) || fbool(hc, &has_cuda)) return -1;
    PyObject *sm = FGET(d, sgpu_metal), *scu = FGET(d, sgpu_cuda), *tm = FGET(d, T_metal), *tcu = FGET(d, T_cuda);
    if (!sm || !scu || !tm || !tcu) return -1;
    const int tsm = ftable(sm), tsc = ftable(scu), ttm = fthru(tm), ttc = fthru(tcu);
    if (tsm < 0 || tsc < 0 || ttm < 0 || ttc < 0) return -1;
    PyObject *table = (has_metal && tsm) ? sm : (has_cuda && tsc) ? scu : NULL;
    PyObject *tg = (has_metal && ttm) ? tm : (has_cuda && ttc) ? tcu : NULL;
    double gv = 0.0, tgv = 1.0;
    if (table && tg) {
        fl |= GPU;
        PyObject *row = _PyDict_GetItem_KnownHash(table, J->Q, J->hQ);
        if (row) {
            if (!fdict(row)) return -1;
            PyObject *b1 = FGET(row, b_1);
            if (!b1) {
                if (J->fq) return -1;
            } else {
                if (ff64(b1, &gv)) return -1;
                fl |= GPU_RATE;
            }
        }
        if (ff64(tg, &tgv)) return -1;
    }
    PyObject *dc = FGET(d, d_avail_cuda), *dm = FGET(d, d_avail_metal);
    if (!dc || !dm) return -1;
    if (has_cuda && dc != Py_None) fl |= CUDA_OK;
    if (dm != Py_None) fl |= METAL_AVAIL | (has_metal ? METAL_OK : 0);
    double fv[10];
    fv[0] = v;
    fv[1] = gv;
    fv[3] = tgv;
    if (ff64(FGET(d, T_cpu), &fv[2]) || ff64(FGET(d, t_kvcpy_cpu), &fv[4]) || ff64(FGET(d, t_kvcpy_gpu), &fv[5]) ||
        ff64(FGET(d, t_ram2vram), &fv[6]) || ff64(FGET(d, t_vram2ram), &fv[7]) || ff64(FGET(d, t_comm), &fv[8]) ||
        ff64(FGET(d, s_disk), &fv[9]))
        return -1;
    int64_t iv[6] = {0, 0, 0, 0, 0, 0};
    if (fi64(FGET(d, d_avail_ram), &iv[0]) || fi64(FGET(d, c_cpu), &iv[1]) || fi64(FGET(d, c_gpu), &iv[2])) return -1;
    if (dc != Py_None && fi64(dc, &iv[3])) return -1; /* dc or 0: an int's value either way */
    if (dm != Py_None && fi64(dm, &iv[4])) return -1;
    if (android) {
        int64_t a1, a2;
        if (fi64(FGET(d, d_bytes_can_swap), &a1) || fi64(FGET(d, d_swap_avail), &a2)) return -1;
        iv[5] = a1 < a2 ? a1 : a2;
    }
    const Py_ssize_t nd = J->nd;
    for (int a = 0; a < 10; ++a) J->f64[a * nd + g] = fv[a];
    for (int a = 0; a < 6; ++a) J->b64[a * nd + g] = (double)iv[a];
    J->cls[g] = (uint8_t)c;
    J->flg[g] = (uint8_t)fl;
    return 0;
}

/* Software prefetch ahead of the read-only pass: the profiles of a large batch are scattered Python
 * objects (the instance, its field dict and the dict's keys object, ~20 value objects, the nested FLOPs
 * tables {Q: {"b_1": v}}), a chain of dependent cache misses per device, so the pass is bound by memory
 * latency. A pipeline of prefetch stages runs ahead of the device being packed, each stage reading only
 * what an earlier stage already brought in and prefetching the next level: PF_OBJ devices ahead the
 * instance, PF_DICT its dict object, PF_KEYS the dict's keys object (the entries), PF_VALS every value
 * object, PF_NEST the nested tables' keys objects, PF_ROW their row dicts. Reads only. */
enum { PF_OBJ = 20, PF_DICT = 15, PF_KEYS = 10, PF_VALS = 6, PF_NEST = 3, PF_ROW = 1 };

static void prefetch_lines(const void *p, int n) {
    const char *c = (const char *)p;
    for (int i = 0; i < n; ++i) __builtin_prefetch(c + 64 * i);
}

static void prefetch_values(PyObject *d) {
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(d, &pos, &k, &v)) __builtin_prefetch(v);
}

/* the nested FLOPs tables of one device dict (values already cached): `keys` prefetches each table's keys
 * object, else (keys cached) its Q row dict and that row's keys object */
static void prefetch_tables(const Job *J, PyObject *d, int keys) {
    PyObject *const t[3] = {FGET(d, scpu), FGET(d, sgpu_metal), FGET(d, sgpu_cuda)};
    for (int a = 0; a < 3; ++a) {
        if (!t[a] || !PyDict_CheckExact(t[a])) continue;
        if (keys) {
            prefetch_lines(((PyDictObject *)t[a])->ma_keys, 3);
        } else {
            PyObject *row = _PyDict_GetItem_KnownHash(t[a], J->Q, J->hQ);
            if (row && PyDict_CheckExact(row)) prefetch_lines(((PyDictObject *)row)->ma_keys, 3);
        }
    }
}

static void *worker(void *arg) {
    const Job *J = (const Job *)arg;
    if (J->nd < 8192) {  /* a small table (one halda_solve): cache-resident, two shallow stages */
        for (Py_ssize_t g = J->lo; g < J->hi && !*J->bail; ++g) {
            if (g + 3 < J->hi) {
                PyObject *d = dev_dict(J->devs[g + 3]);
                if (d) prefetch_values(d);
            }
            PyObject *d = dev_dict(J->devs[g]);
            if (!d || !fdict(d) || fast_dev(J, d, g)) *J->bail = 1;
        }
        return NULL;
    }
    for (Py_ssize_t g = J->lo; g < J->hi && !*J->bail; ++g) {
        if (g + PF_OBJ < J->hi) __builtin_prefetch(J->devs[g + PF_OBJ]);
        if (g + PF_DICT < J->hi) {
#if DICTS_ON_CALLER
            __builtin_prefetch(J->devs[g + PF_DICT]);
#else
            PyObject **dp = _PyObject_GetDictPtr(J->devs[g + PF_DICT]);
            if (dp && *dp) __builtin_prefetch(*dp);
#endif
        }
        if (g + PF_KEYS < J->hi) {
            PyObject *d = dev_dict(J->devs[g + PF_KEYS]);
            if (d) prefetch_lines(((PyDictObject *)d)->ma_keys, 12);
        }
        if (g + PF_VALS < J->hi) {
            PyObject *d = dev_dict(J->devs[g + PF_VALS]);
            if (d) prefetch_values(d);
        }
        if (g + PF_NEST < J->hi) {
            PyObject *d = dev_dict(J->devs[g + PF_NEST]);
            if (d && fdict(d)) prefetch_tables(J, d, 1);
        }
        if (g + PF_ROW < J->hi) {
            PyObject *d = dev_dict(J->devs[g + PF_ROW]);
            if (d && fdict(d)) prefetch_tables(J, d, 0);
        }
        PyObject *d = dev_dict(J->devs[g]);
        if (!d || !fdict(d) || fast_dev(J, d, g)) *J->bail = 1;
    }
    return NULL;
}

static int pack_threads(Py_ssize_t nd) {
    const char *e = getenv("HALDA_PACK_THREADS");
    if (e && *e) return atoi(e);
    if (nd < 8192) return 1;
    cpu_set_t cs;
    int n = 1;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
    return n < 16 ? n : 16;
}

/* 1: packed in parallel; 0: not attempted / given up (the caller packs serially); -1: error set */
static int pack_parallel(PyObject *seq, PyObject *Q, int fq, int fout, double *f64, double *b64, uint8_t *cls,
                         int64_t *off, int64_t *heads, Py_ssize_t nd) {
    (void)fout;
    const Py_ssize_t nf = PySequence_Fast_GET_SIZE(seq);
    int nt = pack_threads(nd);
    if (nt < 1 || !PyUnicode_CheckExact(Q)) return 0;
    const Py_hash_t hQ = PyObject_Hash(Q);
    if (hQ == -1) return -1;
    PyObject **devs = (PyObject **)malloc(sizeof(PyObject *) * (size_t)(nd > 0 ? nd : 1));
    if (!devs) return 0;
    Py_ssize_t g = 0;
    off[0] = 0;
    for (Py_ssize_t f = 0; f < nf; ++f) {
        PyObject *fl = PySequence_Fast_GET_ITEM(seq, f);
        if (!PyList_CheckExact(fl) && !PyTuple_CheckExact(fl)) { free(devs); return 0; }
        const Py_ssize_t M = PySequence_Fast_GET_SIZE(fl);
        if (M == 0 || g + M > nd) { free(devs); return 0; }
        PyObject **items = PySequence_Fast_ITEMS(fl);
        for (Py_ssize_t i = 0; i < M; ++i) {
#if DICTS_ON_CALLER
            if (i + PF_FAR < M) __builtin_prefetch(items[i + PF_FAR]);
            PyObject **dp = _PyObject_GetDictPtr(items[i]); /* under the GIL: may create the dict */
            if (!dp || !*dp || !fdict(*dp)) { free(devs); return 0; }
            devs[g + i] = *dp;
#else
            devs[g + i] = items[i];
#endif
        }
        g += M;
        off[f + 1] = g;
    }
    if (g != nd) { free(devs); return 0; }
    if (nt > 64) nt = 64;
    pthread_t th[64];
    Job jobs[64];
    volatile int bail = 0;
    int started = 0;
    if (nt == 1) { /* small tables: the same read-only pass on the calling thread */
        jobs[0] = (Job){devs, 0, nd, nd, Q, hQ, fq, f64, b64, cls, cls + nd, &bail};
        worker(&jobs[0]);
    }
    for (int t = 0; t < nt && nt > 1; ++t) {
        jobs[t] = (Job){devs, nd * t / nt, nd * (t + 1) / nt, nd, Q, hQ, fq, f64, b64, cls, cls + nd, &bail};
        if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) { bail = 1; break; }
        ++started;
    }
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    free(devs);
    if (bail) return 0;
    const uint8_t *flg = cls + nd;
    for (Py_ssize_t f = 0; f < nf; ++f) { /* kappa's head: the first is_head device, else device 0 */
        heads[f] = off[f];
        for (Py_ssize_t j = off[f]; j < off[f + 1]; ++j)
            if (flg[j] & HEAD) { heads[f] = j; break; }
    }
    return 1;
}

static PyObject *pack(PyObject *self, PyObject *args) {
    (void)self;
    PyObject *fleets, *Q;
    int fq, fout;
    Py_buffer bf, bi, bu, bo, bh;
    if (!PyArg_ParseTuple(args, "OOppw*w*w*w*w*", &fleets, &Q, &fq, &fout, &bf, &bi, &bu, &bo, &bh)) return NULL;
    PyObject *ret = NULL, *seq = PySequence_Fast(fleets, "fleets must be a sequence");
    if (!seq) goto done;
    const Py_ssize_t nf = PySequence_Fast_GET_SIZE(seq);
    const Py_ssize_t nd = bu.len / 2;
    if (bo.len < (Py_ssize_t)(8 * (nf + 1)) || bh.len < (Py_ssize_t)(8 * nf) || bf.len < 80 * nd || bi.len < 48 * nd) {
        PyErr_SetString(PyExc_ValueError, "pack: output buffers too small");
        goto done;
    }
    double *f64 = (double *)bf.buf;
    double *b64 = (double *)bi.buf;
    int64_t *off = (int64_t *)bo.buf, *heads = (int64_t *)bh.buf;
    uint8_t *cls = (uint8_t *)bu.buf, *flg = cls + nd;
    Py_ssize_t g = 0;
    {
        const int par = pack_parallel(seq, Q, fq, fout, f64, b64, cls, off, heads, nd);
        if (par < 0) goto done;
        if (par == 1) {
            g = nd;
            goto checks;
        }
    }
    off[0] = 0;
    for (Py_ssize_t f = 0; f < nf; ++f) {
        PyObject *devs = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, f), "a fleet must be a sequence");
        if (!devs) goto done;
        const Py_ssize_t M = PySequence_Fast_GET_SIZE(devs);
        if (M == 0) {
            Py_DECREF(devs);
            PyErr_SetString(PyExc_IndexError, "list index out of range"); /* the reference's kappa */
            goto done;
        }
        if (g + M > nd) {
            Py_DECREF(devs);
            PyErr_SetString(PyExc_ValueError, "pack: more devices than the buffers hold");
            goto done;
        }
        Py_ssize_t head = 0;
        for (Py_ssize_t i = 0; i < M; ++i) { /* kappa's head: the first is_head device, else device 0 */
            PyObject *d = PyObject_GenericGetDict(PySequence_Fast_GET_ITEM(devs, i), NULL);
            if (!d) { Py_DECREF(devs); goto done; }
            PyObject *h = item(d, is_head);
            const int ih = h ? PyObject_IsTrue(h) : -1;
            Py_DECREF(d);
            if (ih < 0) { Py_DECREF(devs); goto done; }
            if (ih) { head = i; break; }
        }
        heads[f] = g + head;
        for (Py_ssize_t i = 0; i < M; ++i, ++g) {
            PyObject *d = PyObject_GenericGetDict(PySequence_Fast_GET_ITEM(devs, i), NULL);
            if (!d) { Py_DECREF(devs); goto done; }
            int err = -1;
            do {
                PyObject *os = item(d, os_type);
                if (!os) break;
                int c = 3;
                if (PyUnicode_Check(os)) {
                    if (PyUnicode_CompareWithASCIIString(os, "mac_no_metal") == 0) c = 1;
                    else if (PyUnicode_CompareWithASCIIString(os, "mac_metal") == 0) c = 2;
                }
                const int android = PyUnicode_Check(os) && PyUnicode_CompareWithASCIIString(os, "android") == 0;
                PyObject *o;
                int fl = 0, t;
                if (!(o = item(d, is_head)) || (t = PyObject_IsTrue(o)) < 0) break;
                fl |= t ? HEAD : 0;
                if (!(o = item(d, is_unified_mem)) || (t = PyObject_IsTrue(o)) < 0) break;
                fl |= t ? UMA : 0;
                /* alpha reads scpu with f_q; kappa reads the head's scpu with f_out */
                PyObject *sc = item(d, scpu);
                if (!sc) break;
                double v = 0.0;
                if (sc != Py_None && PyObject_IsTrue(sc) > 0 && PyDict_Check(sc)) {
                    PyObject *row = PyDict_GetItemWithError(sc, Q);
                    if (!row && PyErr_Occurred()) break;
                    if (row && row != Py_None) {
                        PyObject *b1 = PyDict_Check(row) ? PyDict_GetItemWithError(row, k_b_1) : NULL;
                        if (!b1 && PyErr_Occurred()) break;
                        if (b1) {
                            if (as_f64(b1, &v)) break;
                            fl |= CPU_RATE;
                        } else if (fq || (fout && i == head)) {
                            no_b1(Q);
                            break;
                        }
                    }
                }
                PyObject *hm = item(d, has_metal), *hc = item(d, has_cuda);
                if (!hm || !hc) break;
                const int has_metal = PyObject_IsTrue(hm), has_cuda = PyObject_IsTrue(hc);
                if (has_metal < 0 || has_cuda < 0) break;
                /* _gpu_table / _pick_T_gpu (dense_common.py:78-97): Metal preferred, truthiness tests */
                PyObject *sm = item(d, sgpu_metal), *scu = item(d, sgpu_cuda), *tm = item(d, T_metal),
                         *tcu = item(d, T_cuda);
                if (!sm || !scu || !tm || !tcu) break;
                PyObject *table = (has_metal && PyObject_IsTrue(sm) > 0) ? sm
                                  : (has_cuda && PyObject_IsTrue(scu) > 0) ? scu : NULL;
                PyObject *tg = (has_metal && PyObject_IsTrue(tm) > 0) ? tm : (has_cuda && PyObject_IsTrue(tcu) > 0) ? tcu : NULL;
                if (PyErr_Occurred()) break;
                double gv = 0.0, tgv = 1.0;
                if (table && tg) {
                    fl |= GPU;
                    int gok = 0;
                    if (rate(table, Q, fq, &gok, &gv)) break;
                    fl |= gok ? GPU_RATE : 0;
                    if (as_f64(tg, &tgv)) break;
                }
                PyObject *dc = item(d, d_avail_cuda), *dm = item(d, d_avail_metal);
                if (!dc || !dm) break;
                if (has_cuda && dc != Py_None) fl |= CUDA_OK;
                if (dm != Py_None) fl |= METAL_AVAIL | (has_metal ? METAL_OK : 0);
                PyObject *const fk[8] = {k_T_cpu, NULL, k_t_kvcpy_cpu, k_t_kvcpy_gpu, k_t_ram2vram, k_t_vram2ram,
                                         k_t_comm, k_s_disk};
                double fv[10];
                fv[0] = v;
                fv[1] = gv;
                fv[3] = tgv;
                int bad = 0;
                for (int a = 0; a < 8 && !bad; ++a) {
                    if (!fk[a]) continue;
                    PyObject *x = item_o(d, fk[a]);
                    bad = !x || as_f64(x, &fv[a == 0 ? 2 : a + 2]);
                }
                if (bad) break;
                int64_t iv[6] = {0, 0, 0, 0, 0, 0};
                PyObject *const ik[3] = {k_d_avail_ram, k_c_cpu, k_c_gpu};
                for (int a = 0; a < 3 && !bad; ++a) {
                    PyObject *x = item_o(d, ik[a]);
                    bad = !x || as_i64(x, &iv[a]);
                }
                if (bad) break;
                if (dc != Py_None && PyObject_IsTrue(dc) > 0 && as_i64(dc, &iv[3])) break; /* dc or 0 */
                if (dm != Py_None && PyObject_IsTrue(dm) > 0 && as_i64(dm, &iv[4])) break;
                if (android) {
                    PyObject *cs = item(d, d_bytes_can_swap), *sa = item(d, d_swap_avail);
                    int64_t a1, a2;
                    if (!cs || !sa || as_i64(cs, &a1) || as_i64(sa, &a2)) break;
                    iv[5] = a1 < a2 ? a1 : a2;
                }
                if (PyErr_Occurred()) break;
                for (int a = 0; a < 10; ++a) f64[a * nd + g] = fv[a];
                for (int a = 0; a < 6; ++a) b64[a * nd + g] = (double)iv[a];
                cls[g] = (uint8_t)c;
                flg[g] = (uint8_t)fl;
                err = 0;
            } while (0);
            Py_DECREF(d);
            if (err) { Py_DECREF(devs); goto done; }
        }
        off[f + 1] = g;
        Py_DECREF(devs);
    }
    if (g != nd) {
        PyErr_SetString(PyExc_ValueError, "pack: device count does not match the buffers");
        goto done;
    }
checks:
    /* FleetTable.check: the reference's ZeroDivisionErrors (alpha: b' / T_cpu; kappa: the head's
     * s_disk and every M1 / M3 device's), after the whole table is packed as there */
    for (Py_ssize_t j = 0; j < nd; ++j) {
        const double sd = f64[9 * nd + j];
        if (f64[2 * nd + j] == 0.0 || (cls[j] != 2 && sd == 0.0)) {
            PyErr_SetString(PyExc_ZeroDivisionError, "float division by zero");
            goto done;
        }
    }
    for (Py_ssize_t f = 0; f < nf; ++f)
        if (f64[9 * nd + heads[f]] == 0.0) {
            PyErr_SetString(PyExc_ZeroDivisionError, "float division by zero");
            goto done;
        }
    Py_INCREF(Py_None);
    ret = Py_None;
done:
    Py_XDECREF(seq);
    PyBuffer_Release(&bf);
    PyBuffer_Release(&bi);
    PyBuffer_Release(&bu);
    PyBuffer_Release(&bo);
    PyBuffer_Release(&bh);
    return ret;
}

/* consts(f64, b64, u8, off, heads, fout, f_out_b1, b_in, b_out, V, out) -> None
 * Per fleet of a packed table, the constant part of obj_value in the reference's own order
 * (halda_p_solver.py:356-357, dense_common.py:211-230): out[0][f] = sum t_comm and out[1][f] = sum xi
 * over the devices from the first (Python's `s = 0; for d in devs: s += ...`), out[2][f] = kappa: the
 * head's four terms, then the M1 devices' and then the M3 devices' RAM-headroom terms in index order.
 * IEEE double arithmetic in that order (built with -ffp-contract=off): the bits of the Python loops.
 * Fleets are independent: large tables are split over the packer's threads (each fleet's sums stay one
 * scalar loop, so the bits do not depend on the split). */
typedef struct {
    const double *f64, *b64;
    const int64_t *off, *heads;
    const uint8_t *cls;
    Py_ssize_t nd, nf, lo, hi;
    int fout;
    double f_out_b1, b_in, b_out, V;
    double *out;
    int bad;
} ConstJob;

static void *consts_range(void *arg) {
    ConstJob *J = (ConstJob *)arg;
    const Py_ssize_t nd = J->nd, nf = J->nf;
    const double *f64 = J->f64, *b64 = J->b64;
    const uint8_t *cls = J->cls, *flg = cls + nd;
    const double *scpu = f64, *Tc = f64 + 2 * nd, *r2v = f64 + 6 * nd, *v2r = f64 + 7 * nd, *tcomm = f64 + 8 * nd,
                 *sd = f64 + 9 * nd;
    const double *ram = b64, *ccpu = b64 + nd, *swap = b64 + 5 * nd;
    double *out = J->out;
    for (Py_ssize_t f = J->lo; f < J->hi; ++f) {
        const int64_t a = J->off[f], b = J->off[f + 1], h = J->heads[f];
        if (a < 0 || b > nd || a > b || h < a || h >= b) {
            J->bad = 1;
            return NULL;
        }
        double t = 0.0, x = 0.0;
        for (int64_t j = a; j < b; ++j) t += tcomm[j];
        for (int64_t j = a; j < b; ++j) x += (r2v[j] + v2r[j]) * ((flg[j] & UMA) ? 0.0 : 1.0);
        double total = 0.0;
        if (J->fout && (flg[h] & CPU_RATE)) total = scpu[h] > 0.0 ? 0.0 + J->f_out_b1 / scpu[h] : 0.0;
        total += (J->b_in / J->V + J->b_out) / Tc[h];
        total += J->b_in / (J->V * sd[h]);
        total += J->b_out / sd[h];
        double tail = 0.0;
        for (int pass = 1; pass <= 3; pass += 2)
            for (int64_t j = a; j < b; ++j)
                if (cls[j] == pass) tail += ((ccpu[j] - ram[j]) - swap[j]) / sd[j];
        out[f] = t;
        out[nf + f] = x;
        out[2 * nf + f] = total + tail;
    }
    return NULL;
}

static int pack_threads(Py_ssize_t nd);

static PyObject *consts(PyObject *self, PyObject *args) {
    (void)self;
    Py_buffer bf, bi, bu, bo, bh, bout;
    int fout;
    double f_out_b1, b_in, b_out, V;
    if (!PyArg_ParseTuple(args, "y*y*y*y*y*pddddw*", &bf, &bi, &bu, &bo, &bh, &fout, &f_out_b1, &b_in, &b_out, &V,
                          &bout))
        return NULL;
    PyObject *ret = NULL;
    const Py_ssize_t nd = bu.len / 2, nf = bh.len / 8;
    if (bf.len < 80 * nd || bi.len < 48 * nd || bo.len < 8 * (nf + 1) || bout.len < 24 * nf) {
        PyErr_SetString(PyExc_ValueError, "consts: buffers too small");
        goto done;
    }
    {
        int nt = pack_threads(nd);
        if (nt < 1) nt = 1;
        if (nt > 64) nt = 64;
        if (nt > nf) nt = (int)(nf > 0 ? nf : 1);
        ConstJob jobs[64];
        pthread_t th[64];
        int started = 0, bad = 0;
        for (int t = 0; t < nt; ++t)
            jobs[t] = (ConstJob){(const double *)bf.buf, (const double *)bi.buf, (const int64_t *)bo.buf,
                                 (const int64_t *)bh.buf, (const uint8_t *)bu.buf, nd, nf, nf * t / nt,
                                 nf * (t + 1) / nt, fout, f_out_b1, b_in, b_out, V, (double *)bout.buf, 0};
        Py_BEGIN_ALLOW_THREADS /* plain arrays only, held by the buffers above */
        for (int t = 1; t < nt; ++t) {
            if (pthread_create(&th[t], NULL, consts_range, &jobs[t]) != 0) break;
            started = t;
        }
        consts_range(&jobs[0]);
        for (int t = started + 1; t < nt; ++t) consts_range(&jobs[t]); /* threads that did not start */
        for (int t = 1; t <= started; ++t) pthread_join(th[t], NULL);
        Py_END_ALLOW_THREADS
        for (int t = 0; t < nt; ++t) bad |= jobs[t].bad;
        if (bad) {
            PyErr_SetString(PyExc_ValueError, "consts: bad offsets");
            goto done;
        }
    }
    Py_INCREF(Py_None);
    ret = Py_None;
done:
    PyBuffer_Release(&bf);
    PyBuffer_Release(&bi);
    PyBuffer_Release(&bu);
    PyBuffer_Release(&bo);
    PyBuffer_Release(&bh);
    PyBuffer_Release(&bout);
    return ret;
}

/* results(cls, x, row, k, obj, off, os_class) -> list
 * The HALDAResult of every fleet of a solved batch (halda._batch_on_gpu), built without Python
 * bytecode per fleet: fleet f's winner row starts at x[row[f]] (-1: no feasible k -> None), w = the
 * rint of its first M entries and n of the next M (int(round(v)): both round half to even), k[f],
 * obj[f], sets = the device indices of class 1 / 2 / 3 in device order (assign_sets,
 * dense_common.py:149-167). Each object is what cls.model_construct(w=..., n=..., k=..., obj_value=...,
 * sets=...) gives: the field dict, its own fields-set, no extra / private state. */
static PyObject *s_dict, *s_fset, *s_extra, *s_priv, *s_w, *s_n, *s_k, *s_obj, *s_sets, *s_m[3], *s_fields_tpl;

/* The interpreter's small ints 0 .. kSmall - 1 (layer counts, device indices), fetched once per results()
 * call: each entry of a list is then one load and an incref, not a PyLong_From* call per entry (that call
 * finds the interpreter state every time; 2 x 64 + 64 entries per fleet). Borrowed: the interpreter keeps
 * its small ints alive. */
enum { kSmall = 257 };
static PyObject *g_small[kSmall];

static int small_ints(void) {
    if (g_small[0]) return 0;
    for (int i = 0; i < kSmall; ++i) {
        PyObject *o = PyLong_FromLong(i);
        if (!o) return -1;
        g_small[i] = o; /* a cached small int: the reference held here is never dropped */
    }
    return 0;
}

static PyObject *int_of(double v) {
    /* int(round(v)), half to even; an integral v (every w / n the solve writes) skips the rounding */
    const double r = fabs(v) < 9.0e18 && v == (double)(long long)v ? v : nearbyint(v);
    if (r >= 0.0 && r < (double)kSmall) {
        PyObject *o = g_small[(int)r];
        Py_INCREF(o);
        return o;
    }
    return fabs(r) < 9.0e18 ? PyLong_FromLongLong((long long)r) : PyLong_FromDouble(r);
}

static PyObject *int_list(const double *v, Py_ssize_t M) {
    PyObject *l = PyList_New(M);
    if (!l) return NULL;
    for (Py_ssize_t i = 0; i < M; ++i) {
        PyObject *o = int_of(v[i]);
        if (!o) { Py_DECREF(l); return NULL; }
        PyList_SET_ITEM(l, i, o);
    }
    return l;
}

static PyObject *index_of(Py_ssize_t i) {
    if (i < kSmall) {
        Py_INCREF(g_small[i]);
        return g_small[i];
    }
    return PyLong_FromSsize_t(i);
}

/* Where model_construct's four stores land in an instance of `cls`: the instance dict's offset and the
 * byte offsets of the three BaseModel slots (member descriptors of object type). Resolved once per class
 * from the type itself; when the class does not have that shape (another pydantic version, a subclass
 * with a custom __setattr__ path for these names) `direct` stays 0 and the generic setattr is used. */
typedef struct {
    PyTypeObject *cls;
    int direct;
    Py_ssize_t fset, extra, priv;
} Slots;
static Slots g_slots;

static Py_ssize_t member_offset(PyTypeObject *cls, PyObject *name) {
    PyObject *d = _PyType_Lookup(cls, name); /* borrowed */
    if (!d || !Py_IS_TYPE(d, &PyMemberDescr_Type)) return -1;
    PyMemberDef *m = ((PyMemberDescrObject *)d)->d_member;
    if ((m->type != T_OBJECT_EX && m->type != T_OBJECT) || (m->flags & READONLY)) return -1;
    return m->offset;
}

static void resolve_slots(PyTypeObject *cls) {
    if (g_slots.cls == cls) return;
    Py_INCREF(cls); /* held: the cached offsets stay keyed to a live type */
    Py_XDECREF(g_slots.cls);
    g_slots.cls = cls;
    g_slots.direct = 0;
    g_slots.fset = member_offset(cls, s_fset);
    g_slots.extra = member_offset(cls, s_extra);
    g_slots.priv = member_offset(cls, s_priv);
    /* model_construct stores through object.__setattr__ (the generic setattr): for a name the type
     * resolves to an object-typed member descriptor that is a store at the member's offset, and for
     * "__dict__" the instance dict slot */
    g_slots.direct = g_slots.fset > 0 && g_slots.extra > 0 && g_slots.priv > 0 && cls->tp_dictoffset > 0;
}

static int put_slot(PyObject *o, Py_ssize_t off, PyObject *v) {
    PyObject **p = (PyObject **)((char *)o + off);
    PyObject *old = *p;
    Py_INCREF(v);
    *p = v;
    Py_XDECREF(old);
    return 0;
}

static PyObject *one_result(PyTypeObject *cls, PyObject *noargs, const double *xr, Py_ssize_t M, long long k, double obj,
                            const uint8_t *cls_row) {
    PyObject *d = NULL, *o = NULL, *fs = NULL, *sets = NULL, *v = NULL;
    if (!(d = PyDict_New())) goto fail;
    if (!(v = int_list(xr, M)) || PyDict_SetItem(d, s_w, v)) goto fail;
    Py_CLEAR(v);
    if (!(v = int_list(xr + M, M)) || PyDict_SetItem(d, s_n, v)) goto fail;
    Py_CLEAR(v);
    if (!(v = PyLong_FromLongLong(k)) || PyDict_SetItem(d, s_k, v)) goto fail;
    Py_CLEAR(v);
    if (!(v = PyFloat_FromDouble(obj)) || PyDict_SetItem(d, s_obj, v)) goto fail;
    Py_CLEAR(v);
    if (!(sets = PyDict_New())) goto fail;
    for (int s = 1; s <= 3; ++s) {
        Py_ssize_t cnt = 0;
        for (Py_ssize_t i = 0; i < M; ++i) cnt += cls_row[i] == s;
        if (!(v = PyList_New(cnt))) goto fail;
        for (Py_ssize_t i = 0, j = 0; i < M; ++i)
            if (cls_row[i] == s) {
                PyObject *ix = index_of(i);
                if (!ix) goto fail;
                PyList_SET_ITEM(v, j++, ix);
            }
        if (PyDict_SetItem(sets, s_m[s - 1], v)) goto fail;
        Py_CLEAR(v);
    }
    if (PyDict_SetItem(d, s_sets, sets)) goto fail;
    Py_CLEAR(sets);
    if (!(fs = PySet_New(s_fields_tpl))) goto fail; /* {w, n, k, obj_value, sets}: a copy, no re-hashing */
    /* object.__new__(cls) and object.__setattr__ of the four slots, as model_construct does */
    if (!(o = PyBaseObject_Type.tp_new(cls, noargs, NULL))) goto fail;
    if (g_slots.cls == cls && g_slots.direct) {
        PyObject **dp = _PyObject_GetDictPtr(o);
        if (!dp) goto fail;
        put_slot(o, (char *)dp - (char *)o, d);
        put_slot(o, g_slots.fset, fs);
        put_slot(o, g_slots.extra, Py_None);
        put_slot(o, g_slots.priv, Py_None);
    } else if (PyObject_GenericSetAttr(o, s_dict, d) || PyObject_GenericSetAttr(o, s_fset, fs) ||
               PyObject_GenericSetAttr(o, s_extra, Py_None) || PyObject_GenericSetAttr(o, s_priv, Py_None)) {
        goto fail;
    }
    Py_DECREF(d);
    Py_DECREF(fs);
    return o;
fail:
    Py_XDECREF(d);
    Py_XDECREF(o);
    Py_XDECREF(fs);
    Py_XDECREF(sets);
    Py_XDECREF(v);
    return NULL;
}

/* sets(os_class) -> {"M1": [...], "M2": [...], "M3": [...]}: the device indices of class 1 / 2 / 3 of
 * one fleet's class row, in device order (assign_sets, dense_common.py:149-167) */
static PyObject *sets_of(PyObject *self, PyObject *args) {
    (void)self;
    Py_buffer bc;
    if (!PyArg_ParseTuple(args, "y*", &bc)) return NULL;
    const uint8_t *cl = (const uint8_t *)bc.buf;
    const Py_ssize_t M = bc.len;
    PyObject *sets = PyDict_New(), *v = NULL;
    if (!sets) goto fail;
    for (int s = 1; s <= 3; ++s) {
        Py_ssize_t cnt = 0;
        for (Py_ssize_t i = 0; i < M; ++i) cnt += cl[i] == s;
        if (!(v = PyList_New(cnt))) goto fail;
        for (Py_ssize_t i = 0, j = 0; i < M; ++i)
            if (cl[i] == s) {
                PyObject *ix = index_of(i);
                if (!ix) goto fail;
                PyList_SET_ITEM(v, j++, ix);
            }
        if (PyDict_SetItem(sets, s_m[s - 1], v)) goto fail;
        Py_CLEAR(v);
    }
    PyBuffer_Release(&bc);
    return sets;
fail:
    Py_XDECREF(sets);
    Py_XDECREF(v);
    PyBuffer_Release(&bc);
    return NULL;
}

static PyObject *results(PyObject *self, PyObject *args) {
    (void)self;
    PyObject *cls;
    Py_buffer bx, br, bk, bo, boff, bc;
    if (!PyArg_ParseTuple(args, "Oy*y*y*y*y*y*", &cls, &bx, &br, &bk, &bo, &boff, &bc)) return NULL;
    PyObject *ret = NULL, *noargs = NULL;
    int gc_was = 0;
    const Py_ssize_t nf = br.len / 8, nx = bx.len / 8, nd = bc.len;
    if (!PyType_Check(cls) || bk.len < 8 * nf || bo.len < 8 * nf || boff.len < 8 * (nf + 1)) {
        PyErr_SetString(PyExc_ValueError, "results: bad arguments");
        goto done;
    }
    /* the cyclic GC paused while the results are made: a few container objects per fleet would trigger
     * collections that walk every object the caller holds (a batch's 262,144 DeviceProfile objects and
     * their dicts: one full collection costs more than building all 4,096 results) */
    gc_was = PyGC_Disable();
    resolve_slots((PyTypeObject *)cls);
    if (!(noargs = PyTuple_New(0)) || !(ret = PyList_New(nf))) goto done;
    const double *x = (const double *)bx.buf, *obj = (const double *)bo.buf;
    const int64_t *row = (const int64_t *)br.buf, *kk = (const int64_t *)bk.buf, *off = (const int64_t *)boff.buf;
    const uint8_t *cl = (const uint8_t *)bc.buf;
    for (Py_ssize_t f = 0; f < nf; ++f) {
        const int64_t a = off[f], M = off[f + 1] - off[f], r = row[f];
        PyObject *o;
        if (r < 0) {
            Py_INCREF(Py_None);
            o = Py_None;
        } else if (a < 0 || M < 0 || a + M > nd || r + 2 * M > nx) {
            PyErr_SetString(PyExc_ValueError, "results: row or device range out of bounds");
            Py_CLEAR(ret);
            goto done;
        } else if (!(o = one_result((PyTypeObject *)cls, noargs, x + r, M, kk[f], obj[f], cl + a))) {
            Py_CLEAR(ret);
            goto done;
        }
        PyList_SET_ITEM(ret, f, o);
    }
done:
    if (gc_was) PyGC_Enable();
    Py_XDECREF(noargs);
    PyBuffer_Release(&bx);
    PyBuffer_Release(&br);
    PyBuffer_Release(&bk);
    PyBuffer_Release(&bo);
    PyBuffer_Release(&boff);
    PyBuffer_Release(&bc);
    return ret;
}

static PyMethodDef methods[] = {{"pack", pack, METH_VARARGS, "Pack fleets of DeviceProfile into the fleet table."},
                                {"consts", consts, METH_VARARGS, "Per-fleet obj_value constants of a packed table."},
                                {"results", results, METH_VARARGS, "HALDAResult per fleet of a solved batch."},
                                {"sets", sets_of, METH_VARARGS, "M1 / M2 / M3 device index lists of a class row."},
                                {NULL, NULL, 0, NULL}};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_fleetpack", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fleetpack(void) {
#define MAKE(n) if (!(k_##n = PyUnicode_InternFromString(#n)) || (h_##n = PyObject_Hash(k_##n)) == -1) return NULL;
    KEYS(MAKE)
#undef MAKE
#define STR(v, s) if (!(v = PyUnicode_InternFromString(s))) return NULL;
    STR(s_dict, "__dict__") STR(s_fset, "__pydantic_fields_set__") STR(s_extra, "__pydantic_extra__")
    STR(s_priv, "__pydantic_private__") STR(s_w, "w") STR(s_n, "n") STR(s_k, "k") STR(s_obj, "obj_value")
    STR(s_sets, "sets") STR(s_m[0], "M1") STR(s_m[1], "M2") STR(s_m[2], "M3")
#undef STR
    {
        PyObject *names = PyTuple_Pack(5, s_w, s_n, s_k, s_obj, s_sets);
        if (!names) return NULL;
        s_fields_tpl = PyFrozenSet_New(names);
        Py_DECREF(names);
        if (!s_fields_tpl) return NULL;
    }
    if (small_ints()) return NULL;
    return PyModule_Create(&mod);
}
