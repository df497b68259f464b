"""ctypes binding of libgibbs_hip.so (include/gibbs_hip.h).

The product path is the HIP library only: if the shared object is missing or
cannot be loaded this module raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import re
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_PATH = PKG_DIR / "libgibbs_hip.so"
HEADER_PATH = REPO_DIR / "include" / "gibbs_hip.h"

GS_OK = 0
GS_E_ARG = 1
GS_E_ROULETTE_OVERRUN = 2
GS_E_OVERFLOW = 3
GS_E_HIP = 4
GS_E_RCCL = 5
GS_E_STATE = 6
GS_E_UNSUPPORTED = 7
UNIQUE_ID_BYTES = 128
SCAN_CERTIFIED = 0
SCAN_EXACT = 1
IPC_HANDLE_BYTES = 64  # include/gibbs_hip.h GS_IPC_HANDLE_BYTES
LOG2_ERR_BUDGET = 2.0 ** -22  # gs_common.h kLog2AbsErr
EXP2_ERR_BUDGET = 2.0 ** -22  # gs_common.h kExp2RelErr
STAT_NAMES = ("exact_rescans", "serial_picks", "rescan_flagged", "rescan_recheck",
              "rescan_total", "rescan_no_lane", "rescan_boundary", "rescan_between_lanes",
              "bg_path", "bg_picks", "live_band", "live_list_full", "live_no_motif",
              "desc_oob")


# Spellings of the tuning fields in the tools' A/B specs (NAME=value)
TUNING_ALIASES = {
    "GS_BLOCKS_PER_CU": "blocks_per_cu_cap", "GS_GROUP_LANES": "group_lanes",
    "GS_SWEEP_WAVES": "sweep_waves", "GS_DNA": "dna_mode", "GS_DNA_G": "dna_G",
    "GS_GRAPH": "graph_mode", "GS_SITE_COOP": "site_coop", "GS_COOP_RATE": "coop_rate",
    "GS_GREEDY_COOP": "motif_coop", "GS_SITE_DT16": "site_dt16",
    "GS_SITE_EXIT_CHUNK": "site_exit_chunk", "GS_SITE_EXIT_RATIO": "site_exit_ratio",
    "GS_GREEDY_EXIT_CHUNK": "greedy_exit_chunk", "GS_GREEDY_EXIT_RATIO": "greedy_exit_ratio",
    "GS_GREEDY_WAVES": "greedy_waves", "GS_MULTI_GREEDY_THREADS": "multi_greedy_threads",
    "GS_MULTI_SPEC_SLOTS": "multi_spec_slots", "GS_GREEDY_SWITCH": "greedy_switch",
    "GS_SITE_SWITCH": "site_switch",
}


def tuning_spec(spec: str) -> dict:
    """'GS_SITE_COOP=0,greedy_waves=4' -> {'site_coop': 0.0, 'greedy_waves': 4.0}."""
    out = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=", 1)
        out[TUNING_ALIASES.get(k, k)] = float(v)
    return out


class GibbsError(RuntimeError):
    """Base error; `.status` is the gs_status, `.index` the failing sequence."""

    def __init__(self, status: int, msg: str, index: int = -1):
        super().__init__(f"[gs_status {status}] {msg}" + (f" (sequence {index})" if index >= 0 else ""))
        self.status = status
        self.index = index


class ArgumentError(GibbsError, ValueError):
    """.NET ArgumentOutOfRangeException / ArgumentException equivalent."""


class RouletteOverrunError(GibbsError, IndexError):
    """The list-index ArgumentException of rouletteWheelSelection (.fs:752)."""


class ChecksumOverflowError(GibbsError, OverflowError):
    """Checked Array.sum overflow (.fs:117)."""


class DeviceError(GibbsError):
    """HIP / RCCL failure (InvalidOperationException in the F# shim)."""


_ERRORS = {
    GS_E_ARG: ArgumentError,
    GS_E_ROULETTE_OVERRUN: RouletteOverrunError,
    GS_E_OVERFLOW: ChecksumOverflowError,
}

_lib = None


def load_library(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libgibbs_hip.so (fails loudly when it is absent)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path).resolve() if path else LIB_PATH
    if not p.exists():
        raise ImportError(
            f"{p} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP path has no CPU fallback)")
    # One HIP runtime per process: when PyTorch is present it must be loaded first so
    # that libgibbs_hip.so binds to torch's libamdhip64.so.7 / librccl (same SONAMEs)
    # instead of pulling /opt/rocm's copies in beside them (two runtimes abort at exit).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(str(p), mode=C.RTLD_LOCAL)
    # (an explicit path may name an older build kept for A/B runs: entry points it
    # lacks stay undeclared there; the shipped library must export every one)
    _declare(lib, strict=path is None)
    if path is None:
        _lib = lib
    return lib


def _declare(lib: C.CDLL, strict: bool = True) -> None:
    vp, i32, i64, u64, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_double
    P = C.POINTER
    sig = {
        "gs_create": (C.c_int, [i32, P(vp)]),
        "gs_destroy": (C.c_int, [vp]),
        "gs_set_tuning": (C.c_int, [vp, C.c_char_p, f64]),
        "gs_get_tuning": (C.c_int, [vp, C.c_char_p, P(f64)]),
        "gs_last_error": (C.c_char_p, [vp]),
        "gs_error_index": (i64, [vp]),
        "gs_version": (C.c_char_p, []),
        "gs_set_sequences": (C.c_int, [vp, vp, vp, i32, vp, i32, i64, i64]),
        "gs_comm_unique_id": (C.c_int, [vp]),
        "gs_comm_init": (C.c_int, [vp, vp, i32, i32]),
        "gs_motif_sweep": (C.c_int, [vp, i32, f64, f64, vp, vp, vp, vp]),
        "gs_state_set_positions": (C.c_int, [vp, i32, vp]),
        "gs_run_sweeps": (C.c_int, [vp, f64, f64, i32, u64, i64]),
        "gs_state_get": (C.c_int, [vp, vp, vp]),
        "gs_prepare_sweeps": (C.c_int, [vp, f64, f64, u64]),
        "gs_synchronize": (C.c_int, [vp]),
        "gs_motif_run": (C.c_int, [vp, i32, f64, f64, i32, u64, i64, vp, vp]),
        "gs_run_greedy": (C.c_int, [vp, f64, f64, i32, P(i32), P(f64)]),
        "gs_motif_greedy": (C.c_int, [vp, i32, f64, f64, i32, vp, vp, P(i32)]),
        "gs_motif_sampling": (C.c_int, [vp, i32, f64, f64, u64, i32, i32, vp, vp, P(i32)]),
        "gs_motif_sweep_multi": (C.c_int, [vp, i32, i32, f64, f64, i32, vp, vp, vp, vp, vp, vp]),
        "gs_motif_greedy_multi": (C.c_int, [vp, i32, i32, f64, f64, i32, i32, vp, vp, vp,
                                            P(i32)]),
        "gs_motif_sampling_multi": (C.c_int, [vp, i32, i32, f64, f64, u64, i32, i32, i32, vp, vp,
                                              vp, P(i32)]),
        "gs_set_fixed_pcv": (C.c_int, [vp, vp]),
        "gs_set_fixed_ppm": (C.c_int, [vp, vp, i32]),
        "gs_site_scan": (C.c_int, [vp, i32, f64, vp, vp, vp]),
        "gs_site_refine": (C.c_int, [vp, i32, f64, i32, i32, vp, vp, P(i32)]),
        "gs_site_sampling": (C.c_int, [vp, i32, f64, u64, i32, i32, vp, vp, vp]),
        "gs_counts": (C.c_int, [vp, i32, vp, vp, vp]),
        "gs_random_starts": (C.c_int, [vp, i32, f64, u64, i32, vp, vp]),
        "gs_best_pwms": (C.c_int, [vp, i32, f64, i32, vp, vp, P(f64), P(i32)]),
        "gs_uniform": (f64, [u64, u64, u64]),
        "gs_stream_sweep": (u64, [u64]),
        "gs_profile_enable": (C.c_int, [vp, i32]),
        "gs_profile_read": (C.c_int, [vp, P(f64), P(i64), P(f64), P(i64)]),
        "gs_profile_region_begin": (C.c_int, [vp]),
        "gs_profile_region_end": (C.c_int, [vp, P(f64)]),
        "gs_profile_region_stop": (C.c_int, [vp]),
        "gs_stats": (C.c_int, [vp, vp, i32]),
        "gs_sweep_kernel_name": (C.c_char_p, [vp]),
        "gs_last_sweep_launch": (C.c_int, [vp, vp]),
        "gs_set_scan_mode": (C.c_int, [vp, i32]),
        "gs_fastmath_check": (C.c_int, [vp, P(f64), P(f64)]),
        "gs_agg_size": (i64, [vp]),
        "gs_agg_download": (C.c_int, [vp, vp]),
        "gs_agg_upload": (C.c_int, [vp, vp]),
        "gs_exchange_handle": (C.c_int, [vp, vp]),
        "gs_exchange_open": (C.c_int, [vp, vp, i32, i32]),
        "gs_exchange_close": (C.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        if not strict and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def header_symbols(header: Path = HEADER_PATH) -> list[str]:
    """Every function declared in include/gibbs_hip.h."""
    text = header.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(gs_\w+)\s*\(", text, re.M)))


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Context:
    """One gs_ctx: one GPU, one shard of the sequences."""

    def __init__(self, device: int = 0, lib_path: str | os.PathLike | None = None,
                 tuning: dict | None = None):
        self.lib = load_library(lib_path)
        h = C.c_void_p()
        st = self.lib.gs_create(int(device), C.byref(h))
        if st != GS_OK:
            raise DeviceError(st, f"gs_create(device={device}) failed")
        self.h = h
        self.n_local = 0
        self.lengths = np.zeros(0, np.int64)
        for k, v in (tuning or {}).items():
            self.set_tuning(k, v)

    def set_tuning(self, name: str, value: float) -> None:
        """Engine tuning field (gs_set_tuning: diagnostics and A/B runs; the results
        never depend on it).  Set before set_sequences."""
        self._check(self.lib.gs_set_tuning(self.h, name.encode(), C.c_double(float(value))))

    def get_tuning(self, name: str) -> float:
        v = C.c_double()
        self._check(self.lib.gs_get_tuning(self.h, name.encode(), C.byref(v)))
        return v.value

    # -- plumbing
    def close(self) -> None:
        if self.h:
            self.lib.gs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int) -> None:
        if st == GS_OK:
            return
        msg = (self.lib.gs_last_error(self.h) or b"").decode(errors="replace")
        idx = int(self.lib.gs_error_index(self.h))
        raise _ERRORS.get(st, DeviceError)(st, msg, idx)

    # -- data
    def set_sequences(self, codes: np.ndarray, offsets: np.ndarray, alphabet: bytes | np.ndarray,
                      n_global: int | None = None, global_offset: int = 0) -> None:
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        alpha = np.frombuffer(bytes(alphabet), np.uint8) if isinstance(alphabet, (bytes, bytearray)) \
            else np.ascontiguousarray(alphabet, dtype=np.uint8)
        n = len(offsets) - 1
        ng = n if n_global is None else int(n_global)
        self._check(self.lib.gs_set_sequences(self.h, _ptr(codes), _ptr(offsets), n, _ptr(alpha),
                                              len(alpha), ng, int(global_offset)))
        self.n_local = n
        self.lengths = np.diff(offsets)
        self._keep = (codes, offsets, alpha)

    def comm_init(self, unique_id: bytes, nranks: int, rank: int) -> None:
        buf = (C.c_uint8 * UNIQUE_ID_BYTES).from_buffer_copy(unique_id)
        self._check(self.lib.gs_comm_init(self.h, buf, int(nranks), int(rank)))

    @staticmethod
    def unique_id() -> bytes:
        lib = load_library()
        buf = (C.c_uint8 * UNIQUE_ID_BYTES)()
        st = lib.gs_comm_unique_id(buf)
        if st != GS_OK:
            raise DeviceError(st, "gs_comm_unique_id failed")
        return bytes(buf)

    # -- hot path
    def motif_sweep(self, W: int, pc: float, cutoff: float, pos_in, u):
        pos_in = np.ascontiguousarray(pos_in, dtype=np.int32)
        u = np.ascontiguousarray(u, dtype=np.float64)
        if pos_in.shape != (self.n_local,) or u.shape != (self.n_local,):
            raise ArgumentError(GS_E_ARG, "pos_in and u need one entry per sequence")
        pos_out = np.empty(self.n_local, np.int32)
        pwms = np.empty(self.n_local, np.float64)
        self._check(self.lib.gs_motif_sweep(self.h, int(W), float(pc), float(cutoff), _ptr(pos_in),
                                            _ptr(u), _ptr(pos_out), _ptr(pwms)))
        return pos_out, pwms

    def set_positions(self, W: int, pos) -> None:
        pos = np.ascontiguousarray(pos, dtype=np.int32)
        self._check(self.lib.gs_state_set_positions(self.h, int(W), _ptr(pos)))

    def run_sweeps(self, pc: float, cutoff: float, n_sweeps: int, seed: int, first_sweep: int = 0):
        self._check(self.lib.gs_run_sweeps(self.h, float(pc), float(cutoff), int(n_sweeps),
                                           int(seed) & (2**64 - 1), int(first_sweep)))

    def prepare_sweeps(self, pc: float, cutoff: float, seed: int) -> None:
        """Capture the sweep-chain graph for the current phase ahead of time."""
        self._check(self.lib.gs_prepare_sweeps(self.h, float(pc), float(cutoff),
                                               int(seed) & (2**64 - 1)))

    def get_state(self):
        pos = np.empty(self.n_local, np.int32)
        pwms = np.empty(self.n_local, np.float64)
        self._check(self.lib.gs_state_get(self.h, _ptr(pos), _ptr(pwms)))
        return pos, pwms

    def synchronize(self) -> None:
        self._check(self.lib.gs_synchronize(self.h))

    def motif_run(self, W, pc, cutoff, n_sweeps, seed, pos, first_sweep=0):
        pos = np.array(pos, dtype=np.int32, copy=True)
        pwms = np.empty(self.n_local, np.float64)
        self._check(self.lib.gs_motif_run(self.h, int(W), float(pc), float(cutoff), int(n_sweeps),
                                          int(seed) & (2**64 - 1), int(first_sweep), _ptr(pos),
                                          _ptr(pwms)))
        return pos, pwms

    def run_greedy(self, pc: float, cutoff: float, max_passes: int = 1000):
        """Greedy refinement of the resident snapshot (.fs:885-929); returns
        (passes, kernel milliseconds)."""
        passes, ms = C.c_int32(0), C.c_double(0.0)
        self._check(self.lib.gs_run_greedy(self.h, float(pc), float(cutoff), int(max_passes),
                                           C.byref(passes), C.byref(ms)))
        return passes.value, ms.value

    def motif_greedy(self, W: int, pc: float, cutoff: float, pos, pwms, max_passes: int = 1000):
        """findBestMotifIndicesWithStartPositions on (pos, pwms) = motifMem; returns
        (pos, pwms, passes)."""
        pos = np.array(pos, dtype=np.int32, copy=True)
        pwms = np.array(pwms, dtype=np.float64, copy=True)
        if pos.shape != (self.n_local,) or pwms.shape != (self.n_local,):
            raise ArgumentError(GS_E_ARG, "pos and pwms need one entry per sequence")
        passes = C.c_int32(0)
        self._check(self.lib.gs_motif_greedy(self.h, int(W), float(pc), float(cutoff),
                                             int(max_passes), _ptr(pos), _ptr(pwms),
                                             C.byref(passes)))
        return pos, pwms, passes.value

    def motif_sampling(self, W: int, pc: float, cutoff: float, seed: int, init_mode: int = 0,
                       max_passes: int = 1000):
        """doMotifSampling (.fs:1034-1038) on the device -> (pos, pwms, greedy passes)."""
        pos = np.empty(self.n_local, np.int32)
        pwms = np.empty(self.n_local, np.float64)
        passes = C.c_int32(0)
        self._check(self.lib.gs_motif_sampling(self.h, int(W), float(pc), float(cutoff),
                                               int(seed) & (2**64 - 1), int(init_mode),
                                               int(max_passes), _ptr(pos), _ptr(pwms),
                                               C.byref(passes)))
        return pos, pwms, passes.value

    # -- motifAmount >= 1 with Positions lists
    def _lists(self, cnt, pos, cap):
        cnt = np.array(cnt, dtype=np.int32, copy=True)
        pos = np.array(pos, dtype=np.int32, copy=True).reshape(self.n_local, cap)
        if cnt.shape != (self.n_local,):
            raise ArgumentError(GS_E_ARG, "cnt needs one entry per sequence")
        return cnt, np.ascontiguousarray(pos)

    def motif_sweep_multi(self, motif_amount: int, W: int, pc: float, cutoff: float, cnt, pos, u,
                          cap: int | None = None):
        """findBestMotifIndicesByWithStartPositions (.fs:935-970) with Positions lists:
        (cnt[n], pos[n, :cnt[n]]) in F# list order -> (cnt, pos[N, cap], pwms)."""
        cap = int(cap or motif_amount)
        cnt, pos = self._lists(cnt, pos, cap)
        u = np.ascontiguousarray(u, dtype=np.float64)
        if u.shape != (self.n_local,):
            raise ArgumentError(GS_E_ARG, "u needs one entry per sequence")
        co = np.empty(self.n_local, np.int32)
        po = np.full((self.n_local, cap), -1, np.int32)
        pw = np.empty(self.n_local, np.float64)
        self._check(self.lib.gs_motif_sweep_multi(self.h, int(motif_amount), int(W), float(pc),
                                                  float(cutoff), cap, _ptr(cnt), _ptr(pos), _ptr(u),
                                                  _ptr(co), _ptr(po), _ptr(pw)))
        return co, po, pw

    def motif_greedy_multi(self, motif_amount: int, W: int, pc: float, cutoff: float, cnt, pos,
                           pwms, max_passes: int = 1000, cap: int | None = None):
        """findBestMotifIndicesWithStartPositions (.fs:885-929) with Positions lists ->
        (cnt, pos[N, cap], pwms, passes)."""
        cap = int(cap or motif_amount)
        cnt, pos = self._lists(cnt, pos, cap)
        pwms = np.array(pwms, dtype=np.float64, copy=True)
        passes = C.c_int32(0)
        self._check(self.lib.gs_motif_greedy_multi(self.h, int(motif_amount), int(W), float(pc),
                                                   float(cutoff), int(max_passes), cap, _ptr(cnt),
                                                   _ptr(pos), _ptr(pwms), C.byref(passes)))
        return cnt, pos, pwms, passes.value

    def motif_sampling_multi(self, motif_amount: int, W: int, pc: float, cutoff: float, seed: int,
                             init_mode: int = 0, max_passes: int = 1000, cap: int | None = None):
        """doMotifSampling (.fs:1034-1038) with any motifAmount ->
        (cnt, pos[N, cap], pwms, greedy passes)."""
        cap = int(cap or motif_amount)
        co = np.empty(self.n_local, np.int32)
        po = np.full((self.n_local, cap), -1, np.int32)
        pw = np.empty(self.n_local, np.float64)
        passes = C.c_int32(0)
        self._check(self.lib.gs_motif_sampling_multi(self.h, int(motif_amount), int(W), float(pc),
                                                     float(cutoff), int(seed) & (2**64 - 1),
                                                     int(init_mode), int(max_passes), cap,
                                                     _ptr(co), _ptr(po), _ptr(pw),
                                                     C.byref(passes)))
        return co, po, pw, passes.value

    def set_fixed_pcv(self, pcv49) -> None:
        """The caller's ProbabilityCompositeVector (49 slots) for the ByPCV / WithBPV
        twins of every entry point; None clears it."""
        if pcv49 is None:
            self._check(self.lib.gs_set_fixed_pcv(self.h, None))
            return
        v = np.ascontiguousarray(pcv49, np.float64)
        if v.shape != (49,):
            raise ArgumentError(GS_E_ARG, "pcv needs the 49 CompositeVector slots")
        self._check(self.lib.gs_set_fixed_pcv(self.h, _ptr(v)))

    def set_fixed_ppm(self, ppm49, W: int | None = None) -> None:
        """The caller's PositionProbabilityMatrix (49 slot rows x W) for the
        initialiser (getMotifsWithBestPWMSOfPPM); None clears it."""
        if ppm49 is None:
            self._check(self.lib.gs_set_fixed_ppm(self.h, None, 0))
            return
        m = np.ascontiguousarray(ppm49, np.float64)
        if m.ndim != 2 or m.shape[0] != 49 or (W is not None and m.shape[1] != W):
            raise ArgumentError(GS_E_ARG, "ppm needs 49 slot rows x motifLength columns")
        self._check(self.lib.gs_set_fixed_ppm(self.h, _ptr(m), int(m.shape[1])))

    def site_scan(self, W: int, pc: float, pos):
        """getBestPWMSs of every target with the others at pos -> (score, pos)."""
        pos = np.ascontiguousarray(pos, dtype=np.int32)
        if pos.shape != (self.n_local,):
            raise ArgumentError(GS_E_ARG, "pos needs one entry per sequence")
        score = np.empty(self.n_local, np.float64)
        out = np.empty(self.n_local, np.int32)
        self._check(self.lib.gs_site_scan(self.h, int(W), float(pc), _ptr(pos), _ptr(score),
                                          _ptr(out)))
        return score, out

    def site_refine(self, W: int, pc: float, shift: int, pos, score, max_passes: int = 1000):
        """shift 0 / -1 / +1: getBestPWMSsWithStartPositions / getLeftShiftedBestPWMSs /
        getRightShiftedBestPWMSs -> (pos, score, passes)."""
        pos = np.array(pos, dtype=np.int32, copy=True)
        score = np.array(score, dtype=np.float64, copy=True)
        if pos.shape != (self.n_local,) or score.shape != (self.n_local,):
            raise ArgumentError(GS_E_ARG, "pos and score need one entry per sequence")
        passes = C.c_int32(0)
        self._check(self.lib.gs_site_refine(self.h, int(W), float(pc), int(shift),
                                            int(max_passes), _ptr(pos), _ptr(score),
                                            C.byref(passes)))
        return pos, score, passes.value

    def site_sampling(self, W: int, pc: float, seed: int, init_mode: int = 0,
                      max_passes: int = 1000):
        """doSiteSampling (.fs:697-701) -> (pos, score, passes of the three stages)."""
        pos = np.empty(self.n_local, np.int32)
        score = np.empty(self.n_local, np.float64)
        passes = np.zeros(3, np.int32)
        self._check(self.lib.gs_site_sampling(self.h, int(W), float(pc), int(seed) & (2**64 - 1),
                                              int(init_mode), int(max_passes), _ptr(pos),
                                              _ptr(score), _ptr(passes)))
        return pos, score, passes

    def counts(self, W: int, pos, A: int):
        pos = np.ascontiguousarray(pos, dtype=np.int32)
        Cm = np.empty(A * W, np.int64)
        T = np.empty(A, np.int64)
        self._check(self.lib.gs_counts(self.h, int(W), _ptr(pos), _ptr(Cm), _ptr(T)))
        return Cm.reshape(A, W), T

    def random_starts(self, W: int, pc: float, seed: int, mode: int = 0):
        score = np.empty(self.n_local, np.float64)
        pos = np.empty(self.n_local, np.int32)
        self._check(self.lib.gs_random_starts(self.h, int(W), float(pc), int(seed) & (2**64 - 1),
                                              int(mode), _ptr(score), _ptr(pos)))
        return score, pos

    # -- host-staged aggregate exchange
    def best_pwms(self, W: int, pc: float, target: int, fcv49, ppm49):
        """getBestPWMSs (.fs:462-479) of local sequence `target` against the caller's
        FrequencyCompositeVector fcv49 (49 int slots) and PPM ppm49 (49 x W)."""
        f = np.ascontiguousarray(fcv49, np.int32).reshape(-1)
        p = np.ascontiguousarray(ppm49, np.float64).reshape(-1)
        if f.size != 49 or p.size != 49 * W:
            raise ArgumentError(GS_E_ARG, "fcv49 needs 49 slots, ppm49 49 x W")
        sc, pos = C.c_double(), C.c_int32()
        self._check(self.lib.gs_best_pwms(self.h, int(W), float(pc), int(target), _ptr(f),
                                          _ptr(p), C.byref(sc), C.byref(pos)))
        return sc.value, pos.value

    def agg_download(self) -> np.ndarray:
        n = int(self.lib.gs_agg_size(self.h))
        out = np.empty(n, np.int64)
        self._check(self.lib.gs_agg_download(self.h, _ptr(out)))
        return out

    def agg_upload(self, agg: np.ndarray) -> None:
        agg = np.ascontiguousarray(agg, np.int64)
        if agg.size != int(self.lib.gs_agg_size(self.h)):
            raise ArgumentError(GS_E_ARG, "aggregate buffer size mismatch")
        self._check(self.lib.gs_agg_upload(self.h, _ptr(agg)))

    # -- in-kernel exchange of the aggregate vector (include/gibbs_hip.h gs_exchange_*)
    def exchange_handle(self) -> bytes:
        """This context's exchange buffer as an IPC handle (64 bytes) for the other ranks."""
        buf = (C.c_uint8 * IPC_HANDLE_BYTES)()
        self._check(self.lib.gs_exchange_handle(self.h, buf))
        return bytes(buf)

    def exchange_open(self, handles: list[bytes], rank: int) -> None:
        """Map every rank's buffer (handles in rank order): the live and long sweeps then
        sum the ranks' aggregate partials in-kernel (no all-reduce after them)."""
        blob = b"".join(handles)
        if len(blob) != IPC_HANDLE_BYTES * len(handles):
            raise ArgumentError(GS_E_ARG, "IPC handles are 64 bytes each")
        arr = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        self._check(self.lib.gs_exchange_open(self.h, arr, len(handles), int(rank)))
        self._xch_open = True

    def exchange_close(self) -> None:
        self._xch_open = False
        self._check(self.lib.gs_exchange_close(self.h))

    def exchange_is_open(self) -> bool:
        return getattr(self, "_xch_open", False)

    # -- measurement
    def profile(self, enable: bool | int) -> None:
        """True: time every launch; k > 1: every k-th (sampling); False: off."""
        k = int(enable) if not isinstance(enable, bool) else (1 if enable else 0)
        self._check(self.lib.gs_profile_enable(self.h, k))

    def region_begin(self) -> None:
        self._check(self.lib.gs_profile_region_begin(self.h))

    def region_stop(self) -> None:
        """Record the region's stop event without waiting (region_end reads it)."""
        self._check(self.lib.gs_profile_region_stop(self.h))

    def region_end(self) -> float:
        """Device milliseconds since region_begin (synchronises)."""
        ms = C.c_double()
        self._check(self.lib.gs_profile_region_end(self.h, C.byref(ms)))
        return ms.value

    def profile_read(self):
        a, b, c, d = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
        self._check(self.lib.gs_profile_read(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return a.value, b.value, c.value, d.value

    def sweep_kernel_name(self) -> str:
        """The kernel the next sweep of the current state runs (measurement records)."""
        return self.lib.gs_sweep_kernel_name(self.h).decode()

    def last_sweep_launch(self) -> dict:
        """The last gs_sweep_kernel launch: its EK (4 = the four-symbol kernel), lanes per
        sequence, wavefronts per workgroup, workgroups (include/gibbs_hip.h)."""
        v = np.zeros(4, np.int32)
        self._check(self.lib.gs_last_sweep_launch(self.h, _ptr(v)))
        return dict(zip(("ek", "gl", "waves", "grid"), (int(x) for x in v)))

    def stats(self) -> dict:
        """Cumulative fallback counters (include/gibbs_hip.h gs_stats)."""
        v = np.zeros(len(STAT_NAMES), np.int64)
        self._check(self.lib.gs_stats(self.h, _ptr(v), len(v)))
        return dict(zip(STAT_NAMES, (int(x) for x in v)))

    def fallbacks(self) -> int:
        """Serial exact roulette picks taken so far."""
        return self.stats()["serial_picks"]

    def set_scan_mode(self, exact: bool) -> None:
        """exact=False: certified binary32 scan (default); True: binary64 for every window."""
        self._check(self.lib.gs_set_scan_mode(self.h, SCAN_EXACT if exact else SCAN_CERTIFIED))

    def fastmath_check(self) -> tuple[float, float]:
        """(max |log2 error|, max relative exp2 error) of the device transcendentals."""
        a, b = C.c_double(), C.c_double()
        self._check(self.lib.gs_fastmath_check(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value


def uniform(seed: int, stream: int, index: int) -> float:
    return float(load_library().gs_uniform(seed & (2**64 - 1), stream, index))


def stream_sweep(t: int) -> int:
    return (1 << 40) | int(t)
