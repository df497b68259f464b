"""ctypes wrapper of oracle/_build/libgibbs_oracle.so.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB = ORACLE_DIR / "_build" / "libgibbs_oracle.so"

GO_OK, GO_E_ARG, GO_E_ROULETTE_OVERRUN, GO_E_OVERFLOW = 0, 1, 2, 3


class OracleError(RuntimeError):
    def __init__(self, code, index=-1):
        super().__init__(f"oracle status {code} at sequence {index}")
        self.code, self.index = code, index


class _Seqs(C.Structure):
    _fields_ = [("codes", C.c_void_p), ("off", C.c_void_p), ("n", C.c_int32),
                ("alphabet", C.c_void_p), ("A", C.c_int32)]


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    return LIB


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        vp, i32, u64, f64 = C.c_void_p, C.c_int32, C.c_uint64, C.c_double
        P = C.POINTER(_Seqs)
        _lib.go_uniform.restype = f64
        _lib.go_uniform.argtypes = [u64, u64, u64]
        _lib.go_uniform_int.restype = i32
        _lib.go_uniform_int.argtypes = [u64, u64, u64, i32]
        _lib.go_log2.restype = f64
        _lib.go_log2.argtypes = [f64]
        _lib.go_sweep_faithful.argtypes = [P, i32, i32, f64, f64, vp, vp, i32, vp, i32, i32, vp, vp,
                                           i32, vp, vp, vp]
        _lib.go_sweep_fast.argtypes = [P, i32, i32, f64, f64, vp, vp, i32, vp, i32, i32, vp, vp,
                                       i32, vp, vp, vp, i32]
        _lib.go_counts.argtypes = [P, i32, vp, vp, i32, vp, vp]
        _lib.go_target_detail.argtypes = [P, i32, f64, vp, vp, i32, i32, vp, vp, vp, vp, vp]
        _lib.go_best_pwms.argtypes = [P, i32, f64, i32, vp, vp, vp, vp]
        _lib.go_random_starts.argtypes = [P, i32, f64, vp, u64, i32, i32, i32, vp, vp]
        _lib.go_sweep_shard.argtypes = [P, C.c_int64, i32, f64, f64, vp, vp, vp, vp, vp, vp, vp]
        _lib.go_greedy.argtypes = [P, i32, i32, f64, f64, vp, vp, i32, vp, i32, vp]
        _lib.go_greedy_fast.argtypes = [P, i32, i32, f64, f64, vp, vp, i32, vp, i32, i32, vp,
                                        vp]
        _lib.go_site_scan.argtypes = [P, i32, f64, vp, i32, i32, vp, vp]
        _lib.go_random_starts_ex.argtypes = [P, i32, f64, vp, u64, i32, i32, i32, vp, vp, vp, vp]
        _lib.go_site_scan_ex.argtypes = [P, i32, f64, vp, i32, i32, vp, vp, vp]
        _lib.go_site_refine_ex.argtypes = [P, i32, f64, i32, vp, vp, vp, i32, vp]
        _lib.go_sweep_pcv.argtypes = [P, i32, f64, f64, vp, vp, vp, vp, vp, vp, vp]
        _lib.go_greedy_pcv.argtypes = [P, i32, f64, f64, vp, vp, vp, i32, vp]
        _lib.go_site_refine.argtypes = [P, i32, f64, i32, vp, vp, i32, vp]
        _lib.go_site_refine_fast.argtypes = [P, i32, f64, vp, vp, i32, C.c_int64, vp, vp]
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Seqs:
    """Holds numpy buffers alive for a go_seqs view."""

    def __init__(self, codes, offsets, alphabet):
        self.codes = np.ascontiguousarray(codes, np.uint8)
        self.off = np.ascontiguousarray(offsets, np.int64)
        self.alpha = np.frombuffer(bytes(alphabet), np.uint8).copy()
        self.n = len(self.off) - 1
        self.A = len(self.alpha)
        self.s = _Seqs(_p(self.codes), _p(self.off), self.n, _p(self.alpha), self.A)

    @property
    def lengths(self):
        return np.diff(self.off)


def _single_to_lists(pos):
    pos = np.asarray(pos, np.int32)
    cnt = (pos >= 0).astype(np.int32)
    return cnt, np.where(pos >= 0, pos, 0).astype(np.int32)


def sweep(seqs: Seqs, W, pc, cutoff, pos, u, faithful=False, t0=0, t1=None, threads=0,
          motif_amount=1, in_cnt=None, in_pos=None, in_cap=1):
    """Returns (pos_out[-1 = []], pwms, margin) for targets [t0,t1); motif_amount=1 form."""
    L = lib()
    n = seqs.n
    t1 = n if t1 is None else t1
    if in_cnt is None:
        in_cnt, in_pos = _single_to_lists(pos)
    in_cnt = np.ascontiguousarray(in_cnt, np.int32)
    in_pos = np.ascontiguousarray(in_pos, np.int32)
    u = np.ascontiguousarray(u, np.float64)
    cap = max(1, motif_amount)
    out_cnt = np.zeros(n, np.int32)
    out_pos = np.full(n * cap, -1, np.int32)
    pwms = np.zeros(n, np.float64)
    margin = np.full(n, np.inf)
    err = C.c_int32(-1)
    if faithful:
        rc = L.go_sweep_faithful(C.byref(seqs.s), motif_amount, W, pc, cutoff, _p(in_cnt),
                                 _p(in_pos), in_cap, _p(u), t0, t1, _p(out_cnt), _p(out_pos), cap,
                                 _p(pwms), _p(margin), C.byref(err))
    else:
        rc = L.go_sweep_fast(C.byref(seqs.s), motif_amount, W, pc, cutoff, _p(in_cnt), _p(in_pos),
                             in_cap, _p(u), t0, t1, _p(out_cnt), _p(out_pos), cap, _p(pwms),
                             _p(margin), C.byref(err), threads)
    if rc:
        raise OracleError(rc, err.value)
    if motif_amount == 1:
        out = np.where(out_cnt > 0, out_pos.reshape(n, cap)[:, 0], -1).astype(np.int32)
        return out, pwms, margin
    return (out_cnt, out_pos.reshape(n, cap)), pwms, margin


def sweep_lists(seqs: Seqs, motif_amount, W, pc, cutoff, cnt, pos, cap, u, faithful=False,
                threads=0):
    """findBestMotifIndicesByWithStartPositions with Positions lists (any motifAmount):
    (cnt[n], pos[n, :cnt[n]]) in F# list order -> (cnt, pos[N, cap_out], pwms)."""
    L = lib()
    n = seqs.n
    cnt = np.ascontiguousarray(cnt, np.int32)
    pos = np.ascontiguousarray(np.asarray(pos, np.int32).reshape(n, cap))
    u = np.ascontiguousarray(u, np.float64)
    oc = max(cap, motif_amount)
    out_cnt = np.zeros(n, np.int32)
    out_pos = np.full((n, oc), -1, np.int32)
    pwms = np.zeros(n, np.float64)
    err = C.c_int32(-1)
    if faithful:
        rc = L.go_sweep_faithful(C.byref(seqs.s), motif_amount, W, pc, cutoff, _p(cnt), _p(pos),
                                 cap, _p(u), 0, n, _p(out_cnt), _p(out_pos), oc, _p(pwms), None,
                                 C.byref(err))
    else:
        rc = L.go_sweep_fast(C.byref(seqs.s), motif_amount, W, pc, cutoff, _p(cnt), _p(pos), cap,
                             _p(u), 0, n, _p(out_cnt), _p(out_pos), oc, _p(pwms), None,
                             C.byref(err), threads)
    if rc:
        raise OracleError(rc, err.value)
    return out_cnt, out_pos, pwms


def greedy_lists(seqs: Seqs, motif_amount, W, pc, cutoff, cnt, pos, cap, pwms, max_passes=1000):
    """findBestMotifIndicesWithStartPositions with Positions lists -> (cnt, pos, pwms, passes)."""
    n = seqs.n
    cnt = np.array(cnt, np.int32, copy=True)
    pos = np.ascontiguousarray(np.array(pos, np.int32, copy=True).reshape(n, cap))
    pw = np.array(pwms, np.float64, copy=True)
    passes = C.c_int32()
    rc = lib().go_greedy(C.byref(seqs.s), motif_amount, W, pc, cutoff, _p(cnt), _p(pos), cap,
                         _p(pw), max_passes, C.byref(passes))
    if rc:
        raise OracleError(rc)
    return cnt, pos, pw, passes.value


def sweep_shard(seqs: Seqs, n_global, W, pc, cutoff, Cglob, Tglob, pos, u):
    """Shard sweep against global aggregates (multi-GPU decomposition model)."""
    Cg = np.ascontiguousarray(Cglob, np.int64).reshape(-1)
    Tg = np.ascontiguousarray(Tglob, np.int64)
    pos = np.ascontiguousarray(pos, np.int32)
    u = np.ascontiguousarray(u, np.float64)
    out = np.zeros(seqs.n, np.int32)
    pw = np.zeros(seqs.n, np.float64)
    err = C.c_int32(-1)
    rc = lib().go_sweep_shard(C.byref(seqs.s), int(n_global), W, pc, cutoff, _p(Cg), _p(Tg),
                              _p(pos), _p(u), _p(out), _p(pw), C.byref(err))
    if rc:
        raise OracleError(rc, err.value)
    return out, pw


def counts(seqs: Seqs, W, pos):
    cnt, p = _single_to_lists(pos)
    Cm = np.zeros(seqs.A * W, np.int64)
    T = np.zeros(seqs.A, np.int64)
    rc = lib().go_counts(C.byref(seqs.s), W, _p(cnt), _p(p), 1, _p(Cm), _p(T))
    if rc:
        raise OracleError(rc)
    return Cm.reshape(seqs.A, W), T


def target_detail(seqs: Seqs, W, pc, pos, n):
    cnt, p = _single_to_lists(pos)
    K = int(seqs.lengths[n]) - W + 1
    bgc = np.zeros(49, np.int64)
    pcv = np.zeros(49, np.float64)
    pwm = np.zeros(seqs.A * W, np.float64)
    S = np.zeros(K, np.float64)
    G = np.zeros(K, np.float64)
    rc = lib().go_target_detail(C.byref(seqs.s), W, pc, _p(cnt), _p(p), 1, n, _p(bgc), _p(pcv),
                                _p(pwm), _p(S), _p(G))
    if rc:
        raise OracleError(rc)
    return dict(bgc=bgc, pcv=pcv, pwm=pwm.reshape(seqs.A, W), S=S, G=G)


def _opt(a):
    return None if a is None else np.ascontiguousarray(a, np.float64)


def random_starts(seqs: Seqs, W, pc, seed=0, mode=0, draws=None, t0=0, t1=None, pcv49=None,
                  ppm49=None):
    """getPWMOfRandomStarts; with pcv49 its ...WithBPV twin, with ppm49 (49 x W slot
    rows) getMotifsWithBestPWMSOfPPM."""
    n = seqs.n
    t1 = n if t1 is None else t1
    score = np.zeros(n, np.float64)
    pos = np.zeros(n, np.int32)
    d = None if draws is None else np.ascontiguousarray(draws, np.int32)
    pcv, ppm = _opt(pcv49), _opt(ppm49)
    rc = lib().go_random_starts_ex(C.byref(seqs.s), W, pc, _p(d), seed & (2**64 - 1), mode, t0,
                                   t1, _p(pcv), _p(ppm), _p(score), _p(pos))
    if rc:
        raise OracleError(rc)
    return score, pos


def best_pwms(seqs: Seqs, W, pc, n, fcv49, ppm):
    fcv = np.ascontiguousarray(fcv49, np.int64)
    ppm = np.ascontiguousarray(ppm, np.float64)
    score, pos = C.c_double(), C.c_int32()
    rc = lib().go_best_pwms(C.byref(seqs.s), W, pc, n, _p(fcv), _p(ppm), C.byref(score),
                            C.byref(pos))
    if rc:
        raise OracleError(rc)
    return score.value, pos.value


def greedy(seqs: Seqs, W, pc, cutoff, pos, pwms, motif_amount=1, max_passes=1000):
    cnt, p = _single_to_lists(pos)
    pw = np.array(pwms, np.float64, copy=True)
    passes = C.c_int32()
    rc = lib().go_greedy(C.byref(seqs.s), motif_amount, W, pc, cutoff, _p(cnt), _p(p), 1, _p(pw),
                         max_passes, C.byref(passes))
    if rc:
        raise OracleError(rc)
    return np.where(cnt > 0, p, -1).astype(np.int32), pw, passes.value


def greedy_fast(seqs: Seqs, W, pc, cutoff, pos, pwms, max_passes=1000, t_limit=0):
    """go_greedy with incremental aggregates (the CPU port); returns
    (pos, pwms, passes, target visits)."""
    cnt, p = _single_to_lists(pos)
    pw = np.array(pwms, np.float64, copy=True)
    passes, visits = C.c_int32(), C.c_int64()
    rc = lib().go_greedy_fast(C.byref(seqs.s), 1, W, pc, cutoff, _p(cnt), _p(p), 1, _p(pw),
                              max_passes, t_limit, C.byref(passes), C.byref(visits))
    if rc:
        raise OracleError(rc)
    return np.where(cnt > 0, p, -1).astype(np.int32), pw, passes.value, visits.value


def site_scan(seqs: Seqs, W, pc, r, t0=0, t1=None, pcv49=None):
    """getBestPWMSs of every target with the others at r (one Jacobi pass)."""
    n = seqs.s.n
    t1 = n if t1 is None else t1
    r = np.ascontiguousarray(r, np.int32)
    score = np.zeros(n, np.float64)
    pos = np.zeros(n, np.int32)
    pcv = _opt(pcv49)
    rc = lib().go_site_scan_ex(C.byref(seqs.s), W, pc, _p(r), t0, t1, _p(pcv), _p(score),
                               _p(pos))
    if rc:
        raise OracleError(rc)
    return score, pos


def site_refine(seqs: Seqs, W, pc, shift, pos, score, max_passes=1000, pcv49=None):
    """shift 0: getBestPWMSsWithStartPositions (.fs:554-585); -1 / +1: the left /
    right shifted passes (.fs:519-550 / .fs:483-517).  Returns (pos, score, passes)."""
    p = np.array(pos, np.int32, copy=True)
    s = np.array(score, np.float64, copy=True)
    passes = C.c_int32()
    pcv = _opt(pcv49)
    rc = lib().go_site_refine_ex(C.byref(seqs.s), W, pc, shift, _p(pcv), _p(p), _p(s), max_passes,
                              C.byref(passes))
    if rc:
        raise OracleError(rc)
    return p, s, passes.value


def site_refine_fast(seqs: Seqs, W, pc, pos, score, max_passes=1000, t_limit=0):
    """getBestPWMSsWithStartPositions (.fs:554-585) with incremental aggregates (the
    timed CPU port).  Returns (pos, score, passes, visits)."""
    p = np.array(pos, np.int32, copy=True)
    s = np.array(score, np.float64, copy=True)
    passes, visits = C.c_int32(), C.c_int64()
    rc = lib().go_site_refine_fast(C.byref(seqs.s), W, pc, _p(p), _p(s), max_passes, t_limit,
                                   C.byref(passes), C.byref(visits))
    if rc:
        raise OracleError(rc)
    return p, s, passes.value, visits.value


def sweep_pcv(seqs: Seqs, W, pc, cutoff, pcv49, pos, u):
    """findBestMotifPositionsWithStartPositionsByPCV (.fs:828-853), motifAmount = 1:
    (pos_out, pwms_out, margin)."""
    n = seqs.n
    pos = np.ascontiguousarray(pos, np.int32)
    u = np.ascontiguousarray(u, np.float64)
    po = np.zeros(n, np.int32)
    pw = np.zeros(n, np.float64)
    mg = np.zeros(n, np.float64)
    err = C.c_int32(-1)
    rc = lib().go_sweep_pcv(C.byref(seqs.s), W, pc, cutoff, _p(_opt(pcv49)), _p(pos), _p(u),
                            _p(po), _p(pw), _p(mg), C.byref(err))
    if rc:
        raise OracleError(rc, err.value)
    return po, pw, mg


def greedy_pcv(seqs: Seqs, W, pc, cutoff, pcv49, pos, pwms, max_passes=1000):
    """findBestMotifPositionsWithStartPositionByPCV (.fs:788-823): (pos, pwms, passes)."""
    p = np.array(pos, np.int32, copy=True)
    pw = np.array(pwms, np.float64, copy=True)
    passes = C.c_int32()
    rc = lib().go_greedy_pcv(C.byref(seqs.s), W, pc, cutoff, _p(_opt(pcv49)), _p(p), _p(pw),
                             max_passes, C.byref(passes))
    if rc:
        raise OracleError(rc)
    return p, pw, passes.value


def uniform(seed, stream, index):
    return lib().go_uniform(seed & (2**64 - 1), stream, index)


def uniform_int(seed, stream, index, k):
    return lib().go_uniform_int(seed & (2**64 - 1), stream, index, k)


def stream_sweep(t):
    return (1 << 40) | int(t)


def stream_init(t):
    return (2 << 40) | int(t)


STREAM_INIT_SHARED = 3 << 40
