# src/distilp/solver/_halda_milp.py  (reference-side binding, INTEGRATION.md path B)
import ctypes, os, numpy as np
from scipy.sparse import csr_array, vstack

_lib = ctypes.CDLL(os.environ.get("HALDA_LIB", "/path/to/distilp_amd/libhalda.so"))
_ctx = ctypes.c_void_p()
assert _lib.halda_init(0, ctypes.byref(_ctx)) == 0

class _Batch(ctypes.Structure):
    _fields_ = [("n_inst", ctypes.c_int32), ("max_cols", ctypes.c_int32), ("max_R1", ctypes.c_int32),
                ("max_tab", ctypes.c_int32), ("max_tab_kc", ctypes.c_int32)] + \
               [(f, ctypes.c_void_p) for f in ("n_cols", "n_rows", "csr_off", "col_off", "row_off", "row_ptr",
                                             "col_idx", "val", "c", "col_lb", "col_ub", "row_lb", "row_ub",
                                             "integrality")] + \
               [("mip_rel_gap", ctypes.c_double), ("mip_abs_gap", ctypes.c_double), ("time_limit", ctypes.c_double),
                ("x0", ctypes.c_void_p), ("y0", ctypes.c_void_p)]

class _Result(ctypes.Structure):
    _fields_ = [(f, ctypes.c_void_p) for f in ("status", "x", "obj_lin", "dual_bound", "gap", "nodes")]

class _Res:  # what solve_fixed_k_milp reads: .success, .x
    def __init__(self, ok, x): self.success, self.x = ok, x

def halda_milp(c, integrality, bounds, constraints, options=None):
    A = csr_array(vstack([csr_array(con.A) for con in constraints]))   # ub rows, then the eq row
    A.sort_indices()
    lo = np.concatenate([np.broadcast_to(con.lb, con.A.shape[0]) for con in constraints]).astype(float)
    hi = np.concatenate([np.broadcast_to(con.ub, con.A.shape[0]) for con in constraints]).astype(float)
    arr = dict(n_cols=np.array([len(c)], np.int32), n_rows=np.array([A.shape[0]], np.int32),
               csr_off=np.zeros(1, np.int64), col_off=np.zeros(1, np.int64), row_off=np.zeros(1, np.int64),
               row_ptr=A.indptr.astype(np.int32), col_idx=A.indices.astype(np.int32), val=A.data.astype(float),
               c=np.asarray(c, float), col_lb=np.asarray(bounds.lb, float), col_ub=np.asarray(bounds.ub, float),
               row_lb=lo, row_ub=hi, integrality=np.asarray(integrality, np.uint8))
    b = _Batch(n_inst=1, **{k: v.ctypes.data for k, v in arr.items()})   # shape summary 0 -> computed by the library
    st = np.zeros(1, np.int32); x = np.zeros(len(c)); f = np.zeros(3); nodes = np.zeros(1, np.int64)
    r = _Result(st.ctypes.data, x.ctypes.data, f[0:].ctypes.data, f[1:].ctypes.data, f[2:].ctypes.data,
                nodes.ctypes.data)
    if _lib.halda_solve_batch(_ctx, ctypes.byref(b), ctypes.byref(r)) != 0:
        raise RuntimeError("libhalda failed")
    return _Res(bool(st[0] == 0), x)
