/*
 * _fleetpack: packs lists of DeviceProfile objects into the flat device-field table of
 * halda_solve_fleets (distilp_amd/solver/fleets.py: fleet_table), in C: one pass over the devices
 * reading each profile's pydantic field dict, no per-field Python bytecode. Same values, flags and
 * exceptions as the Python packer it replaces (which restates dense_common.py:25-126 / :211-230 and
 * the reference's truthiness tests, see fleets.py), so the single-fleet halda_solve path spends
 * microseconds, not a Python loop, before the GPU call.
 *
 *   pack(fleets, Q, fq, fout, f64, i64, u8, off, heads) -> None
 *     fleets  sequence of sequences of DeviceProfile
 *     Q       the model's quantisation key; fq / fout: "b_1" in model.f_q / model.f_out
 *     f64     writable float64 buffer [10][nd] (F64_FIELDS rows), i64: int64 [6][nd], u8: uint8
 *     [2][nd] (os_class row, flags row), off: int64 [n_fleets + 1], heads: int64 [n_fleets]
 *   raises what fleets.fleet_table_py raises, FleetTable.check's ZeroDivisionErrors included
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

enum { HEAD = 1, UMA = 2, CPU_RATE = 4, GPU = 8, GPU_RATE = 16, CUDA_OK = 32, METAL_OK = 64, METAL_AVAIL = 128 };

/* field names, interned once (a lookup hashes nothing: the key objects cache their hash) */
#define KEYS(X) X(os_type) X(is_head) X(is_unified_mem) X(scpu) X(has_metal) X(has_cuda) X(sgpu_metal) \
    X(sgpu_cuda) X(T_metal) X(T_cuda) X(d_avail_cuda) X(d_avail_metal) X(T_cpu) X(t_kvcpy_cpu) X(t_kvcpy_gpu) \
    X(t_ram2vram) X(t_vram2ram) X(t_comm) X(s_disk) X(d_avail_ram) X(c_cpu) X(c_gpu) X(d_bytes_can_swap) \
    X(d_swap_avail) X(b_1)
#define DECL(n) static PyObject *k_##n;
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
    int64_t *i64 = (int64_t *)bi.buf, *off = (int64_t *)bo.buf, *heads = (int64_t *)bh.buf;
    uint8_t *cls = (uint8_t *)bu.buf, *flg = cls + nd;
    Py_ssize_t g = 0;
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
                for (int a = 0; a < 6; ++a) i64[a * nd + g] = iv[a];
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

static PyMethodDef methods[] = {{"pack", pack, METH_VARARGS, "Pack fleets of DeviceProfile into the fleet table."},
                                {NULL, NULL, 0, NULL}};

static struct PyModuleDef mod = {PyModuleDef_HEAD_INIT, "_fleetpack", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fleetpack(void) {
#define MAKE(n) if (!(k_##n = PyUnicode_InternFromString(#n))) return NULL;
    KEYS(MAKE)
#undef MAKE
    return PyModule_Create(&mod);
}
