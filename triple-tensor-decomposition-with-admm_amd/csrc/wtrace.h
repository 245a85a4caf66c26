// Timing experiments only (tools/wtrace.py): per-wave start/end clocks of one
// kernel launch, compiled in with -DTRITD_WTRACE=1 (tools/build_k5_variants.sh).
// Each wave's lane 0 writes {realtime start, realtime end, shader-clock start,
// shader-clock end, HW_ID | XCC_ID << 32} into the translation unit's own
// device array; the last launch overwrites earlier ones.  Off by default: the
// product build has no trace code at all.
#pragma once
#ifndef TRITD_WTRACE
#define TRITD_WTRACE 0
#endif
#if TRITD_WTRACE
#define WT_MAXW 32768
#define WT_DECL(name)                                                                    \
    __device__ unsigned long long name[WT_MAXW * 5];                                     \
    extern "C" int name##_read(unsigned long long* out, int n) {                         \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(name), (size_t)n * 5 * 8) == hipSuccess \
                   ? 0                                                                   \
                   : 1;                                                                  \
    }
#define WT_BEGIN()                                                    \
    const unsigned long long wt_r0 = __builtin_amdgcn_s_memrealtime(); \
    const unsigned long long wt_c0 = __builtin_amdgcn_s_memtime()
#define WT_END(name, wave)                                                                     \
    do {                                                                                       \
        const unsigned long long wt_c1 = __builtin_amdgcn_s_memtime();                         \
        const unsigned long long wt_r1 = __builtin_amdgcn_s_memrealtime();                     \
        const long long wt_w = (wave);                                                         \
        if ((threadIdx.x & 63) == 0 && wt_w >= 0 && wt_w < WT_MAXW) {                          \
            unsigned long long* q = name + 5 * wt_w;                                           \
            q[0] = wt_r0;                                                                      \
            q[1] = wt_r1;                                                                      \
            q[2] = wt_c0;                                                                      \
            q[3] = wt_c1;                                                                      \
            q[4] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |   \
                   ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20)   \
                    << 32);                                                                    \
        }                                                                                      \
    } while (0)
#else
#define WT_BEGIN() \
    do {           \
    } while (0)
#define WT_END(name, wave) \
    do {                   \
    } while (0)
#endif
