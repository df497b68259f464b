// gs_stamps.h — in-kernel phase stamps, diagnostic builds only (make stamps /
// GS_MARKS): never in the shipped library; their run time is not quoted, only the
// phase shares.  A kernel using them declares STAMP_DECL once, marks the end of
// phase i with STAMP(i), and adds its per-wave sums to args.stamps with
// STAMP_FLUSH(count) (needs `lane` and `a.stamps` in scope).
#pragma once
#include <hip/hip_runtime.h>

#include "gs_common.h"

#if defined(GS_STAMPS) && (defined(GS_TL_FINE) || defined(GS_TL_PRO))
// fine timeline marks of gs_sweep_kernel's per-sequence phases (TLF) in place of the
// coarse ones (make variant NAME=tlf VFLAGS="-DGS_STAMPS -DGS_TL_FINE")
#define STAMP_PARAMS
#define STAMP_ARGS
#define STAMP_DECL
#define STAMP(i) \
    do {         \
    } while (0)
#define STAMP_FLUSH(nseq) \
    do {                  \
    } while (0)
#define TLINE(gw, i) \
    do {             \
    } while (0)
#define TL_MARK_(gw, i)                                                               \
    do {                                                                              \
        if ((threadIdx.x & 63) == 0 && a.stamps && (gw) < kTlWaves)                   \
            a.stamps[kStampSlots + (long long)(gw) * kTlMarks + (i)] =                \
                __builtin_amdgcn_s_memrealtime();                                     \
    } while (0)
#ifdef GS_TL_PRO  // prologue marks (TLP) instead of the per-sequence ones
#define TLF(gw, i) \
    do {           \
    } while (0)
#define TLP(gw, i) TL_MARK_(gw, i)
#else
#define TLF(gw, i) TL_MARK_(gw, i)
#endif
#elif defined(GS_STAMPS) && defined(GS_TLINE_ONLY)
// timeline marks alone (make variant NAME=tl VFLAGS="-DGS_STAMPS -DGS_TLINE_ONLY"): the
// per-phase s_memtime stamps and their flush atomics perturb the kernel far more
#define STAMP_PARAMS
#define STAMP_ARGS
#define STAMP_DECL
#define STAMP(i) \
    do {         \
    } while (0)
#define STAMP_FLUSH(nseq) \
    do {                  \
    } while (0)
#define TLINE(gw, i)                                                                  \
    do {                                                                              \
        if ((threadIdx.x & 63) == 0 && a.stamps && (gw) < kTlWaves)                   \
            a.stamps[kStampSlots + (long long)(gw) * kTlMarks + (i)] =                \
                __builtin_amdgcn_s_memrealtime();                                     \
    } while (0)
#elif defined(GS_STAMPS)
// a device function that stamps phases of its own takes STAMP_PARAMS, its caller
// passes STAMP_ARGS
#define STAMP_PARAMS , unsigned long long *st_acc, unsigned long long &st_prev
#define STAMP_ARGS , st_acc, st_prev
#define STAMP_DECL                                \
    unsigned long long st_acc[kStampSlots] = {0}; \
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                              \
    do {                                                      \
        __builtin_amdgcn_sched_barrier(0);                    \
        unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        st_acc[i] += t_ - st_prev;                            \
        st_prev = t_;                                         \
        __builtin_amdgcn_sched_barrier(0);                    \
    } while (0)
#define STAMP_FLUSH(nseq)                                                      \
    do {                                                                       \
        if (lane == 0 && a.stamps) {                                           \
            for (int i_ = 0; i_ < kStampSlots - 1; ++i_)                       \
                atomicAdd(&a.stamps[i_], st_acc[i_]);                          \
            atomicAdd(&a.stamps[kStampSlots - 1], (unsigned long long)(nseq)); \
        }                                                                      \
    } while (0)
// timeline mark i of wavefront gw (global 100 MHz clock, one store by lane 0)
#define TLINE(gw, i)                                                                  \
    do {                                                                              \
        if ((threadIdx.x & 63) == 0 && a.stamps && (gw) < kTlWaves)                   \
            a.stamps[kStampSlots + (long long)(gw) * kTlMarks + (i)] =                \
                __builtin_amdgcn_s_memrealtime();                                     \
    } while (0)
#elif defined(GS_MARKS)
// static instruction accounting (tools/isa_phases.py): phase labels in the ISA
#define STAMP_PARAMS
#define STAMP_ARGS
#define STAMP_DECL
#define STAMP(i) asm volatile(";GSMARK stamp" #i ::: "memory")
#define TLINE(gw, i) asm volatile(";GSMARK tline" #i ::: "memory")
#define STAMP_FLUSH(nseq) \
    do {                  \
    } while (0)
#else
#define STAMP_PARAMS
#define STAMP_ARGS
#define STAMP_DECL
#define STAMP(i) \
    do {         \
    } while (0)
#define TLINE(gw, i) \
    do {             \
    } while (0)
#define STAMP_FLUSH(nseq) \
    do {                  \
    } while (0)
#endif

#ifndef TLF
#define TLF(gw, i) \
    do {           \
    } while (0)
#endif
#ifndef TLP
#define TLP(gw, i) \
    do {           \
    } while (0)
#endif
