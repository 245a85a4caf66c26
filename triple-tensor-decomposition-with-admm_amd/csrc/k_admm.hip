// K5 — the fused ADMM update of one iteration.
//
// Replaces, per element of the shard, the whole chain
//   triple_product(A,B,C)                        triple_product.m:6 (L, never stored)
//   R1, R2, O                                    triple_decomp_ADMM.m:41-43
//   R3, E = sign(R3).*max(|R3|-lambda/muO,0)     :46-47 (soft_threshold.m:2)
//   resL, resO, Y_L, Y_O                         :50-53
//   ||resL||^2, ||resO||^2                       :59
//   T_next = D - O + (1/muL_next)*Y_L            :33 of the NEXT iteration
//   W(ij,k) = sum_t T_next(ij,t) C^(t,k)         mode-1/2 half of update_A/update_B (:78,:86)
// in one pass: reads D, Y_L, Y_O and writes Y_L, Y_O, T (6 N-streams), reads
// and writes E in its compact form (one 256 B slot per 2 KB tile, common.h;
// dense only for overflowed tiles), plus W (N*R/n3 elements).  O is never read inside the loop (E, not O, feeds
// :42), so it is not stored: T_{k+1} = (D - O_k) + Y_L/muL_{k+1} determines it
// and k_o_fixup rebuilds O_k = (D + Y_L/muL_{k+1}) - T_{k+1} when the caller
// asks for it (relative error ~1e-16).
//
// Work decomposition: a wave owns one ij-tile (16 consecutive rows i of one
// fibre j) and walks all its t-tiles of 16.  The big tensors are tile-major
// (common.h): the wave's data is one contiguous stream, each 16x16 tile two
// fully coalesced 1 KB dwordx4 sweeps per tensor, and tile tt+1 is
// prefetched into registers while tile tt is computed.  Per t-tile:
//   L^T(t,ij)  = C^(t,:) . KR(ij,:)^T          RP/4 x v_mfma_f64_16x16x4_f64
//   elementwise update in the MFMA C/D layout  (row t = t0+(l>>4)+4r, col ij = l&15)
//   W^T(k,ij) += C^T(k,t) . T(t,ij)            (RP/16)*4 MFMAs; the C/D register
//                                              of T *is* the B operand (no shuffle)
// W^T accumulates in registers over the whole t range, so W leaves the chip
// once.
//
// Derived Y_O (DY, the default for fp64): with muL == muO (both are opts.mu,
// :16-17, and follow one schedule, :56-57), :43 gives 2 O = (D - L) + E^(k-1)
// + (Y_L - Y_O)/mu, hence from :51-53
//   Y_L^(k) - Y_O^(k) = (Y_L - Y_O) + mu (D - L - 2 O + E^(k)) = mu_k (E^(k) - E^(k-1))
// exactly, for every k (Y_L^(0) = Y_O^(0) = 0).  So Y_O is never stored: the
// K5 of iteration k+1 reads Y_L^(k) and the compact E^(k), E^(k-1) (256 B per
// tile each) and forms Y_O^(k) = Y_L^(k) - mu_k (E^(k) - E^(k-1)) — 4 dense
// N-streams instead of 6.  The rebuilt Y_O differs from MATLAB's by rounding
// only (checked against the restatement on every golden case: L, O, E within
// 1e-11, same k; tests/test_gpu_parity.py holds the GPU to 1e-9).
//
// Parity contract of the elementwise chain.  The file is compiled with
// -ffp-contract=off, so the compiler fuses nothing on its own.  The default
// build (K5_FUSE=1) requests FMAs explicitly in the statements of :41-53 and
// forms O as (R1 + R2)/2 (exact for muL == muO): its values agree with
// MATLAB's separate operators to rounding, not bit for bit, and the tests hold
// it to the tolerances of DESIGN.md §2 (L, O, E 1e-9; errHist 1e-8 relative;
// the same k, including a near-tolerance stop golden).  The norm sums of :59
// use FMAs in both builds: their summation order is this kernel's own (per
// lane, then a fixed-order tree), never MATLAB's, so fusing them costs no
// parity.  -DK5_FUSE=0 builds MATLAB's operator order for the chain itself.
#include "kernels.h"
#include "sweep.h"
#include "wtrace.h"

namespace tritd {

typedef double d4 __attribute__((ext_vector_type(4)));

// Waves per workgroup: exactly one group of 4 ij-tiles (common.h: the TM
// layout interleaves groups of 4 and pads tiles4 to a multiple of 4, so a
// wider workgroup would stream past the allocation; 8 waves measured no
// faster).
static constexpr int K5_WAVES = 4;
#ifndef K5_NT
#define K5_NT 3  // nontemporal hints on the streamed tensors: bit 0 loads, bit 1 stores (round 3, interleaved A/B: nt stores -1.5 % iteration, nt loads a further -0.9 %; round 1 had measured nt loads slower)
#endif
#ifndef K5_FASTDIV
#define K5_FASTDIV 1
#endif
#ifndef K5_SWID
#define K5_SWID 1
#endif
#ifndef K5_CSIGN
#define K5_CSIGN 2
#endif
#ifndef K5_IBAL
#define K5_IBAL 1
#endif
#ifndef K5_KRLDS
#define K5_KRLDS 0
#endif
#ifndef K5_LSPLIT
#define K5_LSPLIT 1
#endif
#ifndef K5_EXP
#define K5_EXP 0  // timing experiments only (tools/): drop parts of the t-tile work
#endif
#ifndef K5_FUSE
#define K5_FUSE 1  // fused multiply-adds in the elementwise chain (see the t-tile body)
#endif
#ifndef K5_DNBR
#define K5_DNBR 0  // dense-tile override of the decoded E as a branch (1) or selects (0)
#endif
#ifndef K5_PIPE
#define K5_PIPE 0  // L of t-tile tt+1 computed during t-tile tt (triple-buffered C^ slices)
#endif
#ifndef K5_PROF
#define K5_PROF 0  // timing experiments only: s_memtime phase profile of the t-walk (tools/k5_prof.py)
#endif
#ifndef K5_BUF
#define K5_BUF 1  // streams and compact-E slots through wave-based buffer descriptors (see load; interleaved A/B: K5 -0.6 to -1.0 %)
#endif
#ifndef K5_WPE
#define K5_WPE 2  // waves per SIMD at RP <= 64 (one wave: 1.243 vs 0.998 ms, round 3)
#endif

#if TRITD_WTRACE
WT_DECL(g_wt_k5)
#endif
#if K5_PROF
// phase clocks of the t-walk summed over waves: [0..7] phases, [8] steps
__device__ unsigned long long g_k5prof[16];
#define K5_PT(n)                                          \
    do {                                                  \
        __builtin_amdgcn_sched_barrier(0);                \
        const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
        if ((n) > 0) pacc[(n) - 1] += t_ - plast;         \
        plast = t_;                                       \
        __builtin_amdgcn_sched_barrier(0);                \
    } while (0)
#else
#define K5_PT(n) \
    do {         \
    } while (0)
#endif

__device__ __forceinline__ double matlab_sign(double x) {
    // sign(): 1 / -1 / 0 (also for -0), NaN stays NaN; selects only, no
    // branches (a divergent branch would break the K5 loop's exact vmcnt waits)
    const double s = x == 0.0 ? 0.0 : __builtin_copysign(1.0, x);
    return __builtin_isnan(x) ? x : s;
}

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2v ld2(const d2v* p) {
    if (K5_NT & 1) return __builtin_nontemporal_load(p);
    return *p;
}
__device__ __forceinline__ void st2(d2v v, d2v* p) {
    if (K5_NT & 2)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// --- compact E (common.h: CE) -------------------------------------------
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
constexpr int OOB = 0x40000000;  // buffer offset past any range: the access is dropped (loads give 0)

// buffer descriptor of `bytes` bytes at p (p made wave-uniform explicitly, so
// the descriptor lives in SGPRs without a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, int bytes) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, bytes,
                                             0x00020000);
}
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// bit `lane` of a wave-uniform mask: the mask itself as the lane condition
// (one v_cndmask per use instead of a 64-bit shift, and and compare)
__device__ __forceinline__ bool lane_bit(uint64_t m, int lane) {
#if K5_IBAL
    (void)lane;
    return __builtin_amdgcn_inverse_ballot_w64(m);
#else
    return (m >> lane) & 1;
#endif
}
// Compact-E slot (common.h: CE): words 0..26 the nonzero values, bytes
// CE_IDX_BYTE + q their in-tile positions 64 w + l (element w of lane l, the
// register order), word CE_CNT_WORD the count (low dword; all ones: dense).
// A lane holds slot word lane & 31.
__device__ __forceinline__ bool ce_is_dense(double sv) {
    return (uint32_t)__builtin_amdgcn_readlane(__double2loint(sv), CE_CNT_WORD) == 0xFFFFFFFFu;
}
// This lane's 4 elements (register order) of the tile whose slot word is sv,
// through the wave's LDS tile image img (CE_IMG doubles, all zero on entry and
// on return): lane q < count writes its own value (word q) at its position,
// every lane reads its four, and the writers zero their position again.  No
// mask walk: the position byte comes from one lane-constant ds_bpermute pair.
// Returns true for a dense (overflowed) tile, whose values are in E instead.
__device__ __forceinline__ bool ce_decode(double sv, int lane, double* img, double (&e)[4]) {
    const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane(__double2loint(sv), CE_CNT_WORD);
    const int q = lane & 31;
    const int src = (CE_IDX_BYTE / 8 + (q >> 3)) << 2;  // slot word holding byte q (lane-constant)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, __double2loint(sv));
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, __double2hiint(sv));
    const int pos = (int)__builtin_amdgcn_ubfe((q & 4) ? hi : lo, 8 * (q & 3), 8);
    // cnt <= CE_CAP < 32 unless dense (all ones), so lanes >= 32 never write
    const int at = ((uint32_t)lane < cnt && cnt <= (uint32_t)CE_CAP) ? pos : 256 + lane;
    img[at] = sv;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int w = 0; w < 4; ++w) e[w] = img[64 * w + lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    img[at] = 0.0;
    return cnt == 0xFFFFFFFFu;
}
// Store this lane's 4 elements of E (register order) as the tile's slot at
// (rs, soff), or densely into E2 at d2v offset o when they do not fit.  cs:
// the wave's 96-double LDS scratch (slot image + a junk area for the zeros).
// Branch-free: a branch here makes the compiler's vmcnt waits drain the
// prefetch.
__device__ __forceinline__ void ce_encode_r(const double (&En)[4], int lane, double* cs,
                                            __amdgpu_buffer_rsrc_t rs, int soff, d2v* E2, int64_t o,
                                            unsigned& ndense);
__device__ __forceinline__ void ce_encode(const double (&En)[4], int lane, double* cs, double* CE,
                                          int64_t sb, d2v* E2, int64_t o,
                                          unsigned& ndense) {
    ce_encode_r(En, lane, cs, wave_rsrc(CE + sb, CE_SLOT * 8), 0, E2, o, ndense);
}
// the same with the slot's buffer descriptor and scalar offset given
__device__ __forceinline__ void ce_encode_r(const double (&En)[4], int lane, double* cs,
                                            __amdgpu_buffer_rsrc_t rs, int soff, d2v* E2, int64_t o,
                                            unsigned& ndense) {
    uint64_t nz[4];
    int cnt = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        nz[w] = __ballot(En[w] != 0.0);
        cnt += __builtin_popcountll(nz[w]);
    }
    const int l = lane & 31;
    const bool dense = cnt > CE_CAP;
    // slot image: zeros (lanes >= 32 zero their junk word), then the values
    // and their position bytes, then the count
    cs[lane < 32 ? lane : lane + 32] = 0.0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    unsigned char* cb = reinterpret_cast<unsigned char*>(cs);
    int pre = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        // (a dense tile's image is not used: its values and bytes go to the
        // lane's junk word)
        const bool bit = !dense && lane_bit(nz[w], lane);
        const int at = pre + lanes_below(nz[w]), away = 32 + lane;
        cs[bit ? at : away] = En[w];
        cb[bit ? CE_IDX_BYTE + at : 8 * away + w] = (unsigned char)(64 * w + lane);
        pre += __builtin_popcountll(nz[w]);
    }
    if (lane == 0) cs[CE_CNT_WORD] = __longlong_as_double(dense ? 0xFFFFFFFFll : (long long)cnt);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const double v = cs[l];
    // the dense tile only when it does not fit (wave-uniform, rare: a branch
    // with stores only leaves the common path's waits exact), the slot from
    // lanes 0..31 (an out-of-range offset drops the rest)
    if (dense) {
        E2[o] = d2v{En[0], En[1]};
        E2[o + 64] = d2v{En[2], En[3]};
        ++ndense;  // wave-uniform; one atomic per wave at the end (a per-tile
                   // atomic on one counter serialised: 17 -> 53 ms once E turned dense)
    }
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rs, lane < 32 ? l * 8 : OOB,
                                          soff, 0);
}

// Two waves per SIMD (VGPRs + AGPRs <= 256): at one wave per SIMD the
// streams do not keep enough bytes in flight (measured +6 % K5 time).
// DE (dense-E mode, DY only): E^(k), E^(k-1) and E^(k+1) live densely in the
// tile-major E buffers for every tile — no compact slots are read, decoded,
// encoded or written.  The session switches to it once E has turned dense
// (video-like data: every tile overflows its slot and the compact form only
// adds the slot traffic and the decode/encode work; solver.cpp run()).
template <int RP, bool PRO, bool DY, bool DE = false>
__global__ __launch_bounds__(64 * K5_WAVES) __attribute__((amdgpu_waves_per_eu(RP >= 128 ? 1 : K5_WPE, K5_WPE)))
void k5_fused(K5Args a) {
    static_assert(!DE || (DY && !PRO), "k5_fused: dense-E mode is a derived-Y_O update");
    if (*a.stop) return;
    // side job: workgroup 0 runs the R x R solve of the next update_A
    // (sweep.h) beside the walk, so no second stream is needed for it
    constexpr bool SIDE_OK = !PRO && RP <= 64;
    const int side = SIDE_OK ? a.side.on : 0;
    if constexpr (SIDE_OK) {
        if (side && blockIdx.x == 0) {
            __shared__ double srow[2 * 4 * 64 + RP];
            side_solve<RP>(a.side, srow, srow + 2 * 4 * 64);
            return;
        }
    }
    // workgroup wgi = chunk c of the t-walk (a.tsplit chunks; 1 unless the
    // problem has too few ij-tiles to fill the GPU, k5_tsplit) x group bid of
    // 4 ij-tiles
    const int64_t wgi = (int64_t)blockIdx.x - side;
    const int64_t ngrp = (a.tiles + K5_WAVES - 1) / K5_WAVES;
    const int64_t chunk = wgi / ngrp;
    const int64_t bid = wgi - chunk * ngrp;  // this workgroup's group of ij-tiles
    WT_BEGIN();
    constexpr int KS = RP / 4;   // MFMA K-steps for L
    constexpr int MT = RP / 16;  // k-tiles of W
    constexpr int LDC = RP + 16; // row stride of the [t][k] C^ slice (2*LDC = 32 mod 64: no bank conflicts)
    // row stride of the [k][t] slice: odd, so the staging writes (32 lanes of
    // one t, k = 0, 2, .., 62) fall on distinct banks (stride 16 put them all
    // on one: 16-way conflicts, ~45 % of K5's LDS cycles); the L-operand
    // reads then share one bank pair between two lanes (3 LDS cycles, not 2)
    constexpr int SK = 17;
    const int lane = threadIdx.x & 63;
    // wave-uniform in SGPRs: every tile base below becomes scalar address math
    // (K5 is VALU-issue-bound)
    const int wid = K5_SWID ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : (threadIdx.x >> 6);
    const int il = lane & 15;
    const int tg = lane >> 4;
    const int64_t tile = bid * K5_WAVES + wid;
    const bool active = tile < a.tiles;
    const int64_t qper = a.n1p >> 4;
    const int64_t j = active ? tile / qper : 0;
    const int64_t i = active ? ((tile - j * qper) << 4) + il : 0;
    const int64_t ntt = a.ntt;
    const int64_t t0 = chunk * ntt / a.tsplit, t1 = (chunk + 1) * ntt / a.tsplit;  // this chunk's t-tiles
    // this lane's d2v slot of pair p in t-tile tt: tm_tile_base(tile, tt)/2 + 64p + lane

    // C^ rows of one t-tile, staged once per workgroup:
    //   sCT[k][SK]  (L operand: C^(t0+l&15, 4s+(l>>4)))
    //   sC [16][LDC] (W operand: C^(t0+4r+(l>>4), 16m+(l&15)))
    // PIPE: the L MFMAs of t-tile tt+1 run during t-tile tt, beside its
    // elementwise chain (they depend only on C^ and the Khatri-Rao operand),
    // so a wave always has independent MFMA work to issue while its VALU
    // chain waits on latencies.  Slices tt (W), tt+1 (L) and the one being
    // staged (tt+2) are live at once: three buffers.  Otherwise the L chain
    // heads each t-tile and two buffers suffice.
    constexpr bool PIPE = K5_PIPE && !PRO && RP <= 64;
    constexpr int NB = PIPE ? 3 : 2;
    __shared__ double sCT[NB][RP * SK];
    __shared__ double sC[NB][16 * LDC];
    // per-wave 16x16 transpose buffer for T (stored in the M3 B-operand order)
    __shared__ double tsm[K5_WAVES][16 * 17];
    double* ts = tsm[wid];
    // Rotated t-walk: resident workgroups start at different t-tiles so that
    // their concurrent streams do not advance in lockstep 64 KB apart (HBM
    // channel hot-spotting).  Any fixed order is deterministic.
    const int64_t rot = a.rot ? (bid * 7) % ntt : 0;
    auto phys = [&](int64_t tt) { int64_t x = tt + rot; return x >= ntt ? x - ntt : x; };
    // Staging is split so that its global loads are issued before the tile
    // prefetch and its LDS writes come after this t-tile's compute: vmcnt is
    // in-order, so a wait on a load issued after the prefetch would also wait
    // for the prefetch (measured: the prefetch was serialized every t-tile).
    constexpr int SP = 16 * RP / 2;                 // (v0,v1) pairs per slice
    constexpr int NS = (SP + 64 * K5_WAVES - 1) / (64 * K5_WAVES);
    d2v sv[NS];
#if K5_BUF
    // C^ slices through one descriptor: slice tt at a scalar offset
    const __amdgpu_buffer_rsrc_t rCh = wave_rsrc(a.Ch, (int)(a.n3p * RP * 8));
#endif
    auto stage_load = [&](int64_t tt) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5_WAVES;
            if (SP % (64 * K5_WAVES) == 0 || e < SP) {
#if K5_BUF
                sv[q] = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rCh, 16 * e, (int)(phys(tt) * 16 * RP * 8), 0));
#else
                sv[q] = *reinterpret_cast<const d2v*>(a.Ch + (phys(tt) << 4) * RP + 2 * e);
#endif
            }
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5_WAVES;
            if (SP % (64 * K5_WAVES) == 0 || e < SP) {
                const int row = (2 * e) / RP, k = (2 * e) % RP;
                sC[buf][row * LDC + k] = sv[q][0];
                sC[buf][row * LDC + k + 1] = sv[q][1];
                sCT[buf][k * SK + row] = sv[q][0];
                sCT[buf][(k + 1) * SK + row] = sv[q][1];
            }
        }
    };
    auto stage = [&](int64_t tt, int buf) {
        stage_load(tt);
        stage_store(buf);
    };

#if K5_KRLDS
    // the Khatri-Rao operand lives in LDS (16 doubles per lane, 8 KB per wave):
    // 32 VGPRs fewer for the t-walk (K5 runs at the 256-VGPR, 2-wave limit)
    __shared__ double krm[K5_WAVES][KS * 64];
    double* krs = krm[wid];
    if (!PRO) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + tg;
            krs[s * 64 + lane] =
                active ? a.Ah[j * a.ahj + i * RP + k] * a.Bh[j * a.bhj + k] : 0.0;  // CP or Qi (kernels.h)
        }
    }
#define KR(s) krs[(s) * 64 + lane]
#else
    double kr[KS];
    if (!PRO) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + tg;
            kr[s] = active ? a.Ah[j * a.ahj + i * RP + k] * a.Bh[j * a.bhj + k] : 0.0;  // CP or Qi (kernels.h)
        }
    }
#define KR(s) kr[s]
#endif
    d4 wacc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) wacc[m] = d4{0.0, 0.0, 0.0, 0.0};

    double ssL = 0.0, ssO = 0.0;
    unsigned ndense = 0;  // E tiles of this wave stored densely (wave-uniform)
    const IterScalars sc = a.s;
    const d2v* D2 = reinterpret_cast<const d2v*>(a.D);
    d2v* O2 = reinterpret_cast<d2v*>(a.O);
    d2v* E2 = reinterpret_cast<d2v*>(a.E);
    d2v* Ep2 = reinterpret_cast<d2v*>(a.Ep);     // DY: E^(k-1) dense tiles, E^(k+1) destination
    d2v* Eout2 = DY ? Ep2 : E2;
    [[maybe_unused]] double* CEout = DY ? a.CEp : a.CE;
    d2v* YL2 = reinterpret_cast<d2v*>(a.YL);
    d2v* YO2 = reinterpret_cast<d2v*>(a.YO);
    d2v* T2 = reinterpret_cast<d2v*>(a.T);

    // Two register sets: x[0] = D, x[1] = Y_L, x[2] = Y_O (PRO: O), ed = the
    // tile's dense E (only meaningful for an overflowed tile) and ce = the
    // lane's word of a compact-E slot.  The t-walk is unrolled by two so that
    // the sets alternate by name: a copy cur = next would make the compiler
    // wait for the prefetch at the copy.  Slots are loaded two tiles ahead,
    // so when tile tt+1's batch is issued it is already known whether that
    // tile is dense; its dense E load is issued either way, as a buffer load
    // whose offset is out of range unless it is (no traffic), so the walk has
    // no branches at all (a join
    // makes the compiler's in-order vmcnt waits conservative, i.e. it waits
    // on the batch it just issued).  Nothing depends on `active` either (a
    // wave past the last tile streams the zero-filled group padding).
    // DY: x[2] is unused (Y_O is rebuilt); edp/cep hold E^(k-1) like ed/ce
    struct Regs {
        d2v x[3][2];
        d2v ed[2];
        double ce;
        d2v edp[2];
        double cep;
        d4 l;  // PIPE: L of this t-tile, computed during the previous one
    };
    __shared__ double csm[K5_WAVES][96];
    double* cs = csm[wid];
    // compact-E decode images (ce_decode), zero between uses: one per slot
    // stream (E^(k), E^(k-1) with dy) where the LDS allows, else shared
    constexpr int NIMG = (DE || PRO) ? 0 : ((DY && RP <= 64) ? 2 : 1);
    __shared__ double cimg[NIMG > 0 ? K5_WAVES * NIMG : 1][CE_IMG];
    double* img = cimg[NIMG > 0 ? wid * NIMG : 0];
    double* imgp = cimg[NIMG > 1 ? wid * NIMG + 1 : (NIMG > 0 ? wid * NIMG : 0)];
    if constexpr (NIMG > 0) {
        for (int e = lane; e < NIMG * CE_IMG; e += 64) img[e] = 0.0;  // (imgp follows img)
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    // every __shared__ array of this kernel, in bytes (160 KiB per CU; RP =
    // 256 at one wave per SIMD is the largest: ~147 KB)
    constexpr size_t LDS_BYTES =
        sizeof(double) * (NB * RP * SK + NB * 16 * LDC + K5_WAVES * 16 * 17 + K5_WAVES * 96 + (NIMG > 0 ? K5_WAVES * NIMG : 1) * CE_IMG +
                          2 * K5_WAVES + (K5_KRLDS ? K5_WAVES * KS * 64 : 0));
    static_assert(LDS_BYTES <= 160 * 1024, "k5_fused: LDS over the 160 KiB of a CU");
#if K5_BUF
    // D, Y_L, T through buffer descriptors based at this wave's first tile:
    // the t-tile offset is a scalar (soffset), the lane offset a constant
    // VGPR, so the streams need no per-step 64-bit address VALU
    // (tm_tile_base = wave base + tt * 1024 doubles)
    const int64_t wbase = tm_tile_base(tile, 0, ntt);
    const int wbytes = (int)(ntt * 8192);
    const __amdgpu_buffer_rsrc_t rD = wave_rsrc(a.D + wbase, wbytes);
    const __amdgpu_buffer_rsrc_t rYL = wave_rsrc(a.YL + wbase, wbytes);
    const __amdgpu_buffer_rsrc_t rT = wave_rsrc(a.T + wbase, wbytes);
    const int vlane = lane * 16;
    constexpr int BAUX = K5_NT ? 2 : 0;  // nontemporal
    auto bld = [&](__amdgpu_buffer_rsrc_t r, int64_t tt, int p) {
        return __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(
                                            r, vlane + 1024 * p, (int)(phys(tt) * 8192), BAUX));
    };
    auto bst = [&](d2v v, __amdgpu_buffer_rsrc_t r, int64_t tt, int p) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), r, vlane + 1024 * p,
                                               (int)(phys(tt) * 8192), BAUX);
    };
#endif
    auto load = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tm_tile_base(tile, phys(tt), ntt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#if K5_BUF
            if (!PRO && DY) {
                nx.x[0][p] = bld(rD, tt, p);
                nx.x[1][p] = bld(rYL, tt, p);
                continue;
            }
#endif
            nx.x[0][p] = ld2(D2 + o + 64 * p);
            nx.x[1][p] = ld2(YL2 + o + 64 * p);
            if (PRO || !DY) nx.x[2][p] = ld2((PRO ? O2 : YO2) + o + 64 * p);
        }
    };
    auto load_dense = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tm_tile_base(tile, phys(tt), ntt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p) nx.ed[p] = E2[o + 64 * p];
    };
    auto load_dense_p = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tm_tile_base(tile, phys(tt), ntt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p) nx.edp[p] = Ep2[o + 64 * p];
    };
#if K5_BUF
    // compact-E slots: 4 slots (1 KB) per t-tile from the wave's first one
    const int64_t wslot = (tm_tile_base(tile, 0, ntt) >> 8) * CE_SLOT;
    const __amdgpu_buffer_rsrc_t rCE = wave_rsrc(a.CE + wslot, (int)(ntt * 1024));
    const __amdgpu_buffer_rsrc_t rCEp = wave_rsrc(a.CEp + wslot, (int)(ntt * 1024));
    const int vslot = (lane & 31) * 8;
#endif
    auto load_slot = [&](int64_t tt, Regs& rx) {
        if constexpr (DE) return;
        const int64_t t2 = tt < ntt ? tt : ntt - 1;  // clamped: no branch
#if K5_BUF
        if (!PRO) {
            const int so = (int)(phys(t2) * 1024);
            rx.ce = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rCE, vslot, so, 0));
            if (DY) rx.cep = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rCEp, vslot, so, 0));
            return;
        }
#endif
        const int64_t so = (tm_tile_base(tile, phys(t2), ntt) >> 8) * CE_SLOT + (lane & 31);
        rx.ce = a.CE[so];
        if (DY) rx.cep = a.CEp[so];
    };
    // one t-tile: cx holds its data; if `pf`, tile tt+1 is prefetched into nx
    // and its C^ slice staged into buffer buf^1
    // L^T(t, ij) of the slice in sCT[b]: KS dependent MFMAs
    auto l_mfma = [&](int b) {
        const double* cT = sCT[b];
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        if (!(K5_EXP & 1))
#pragma unroll
            for (int s = 0; s < KS; ++s) acc = mfma4(cT[(4 * s + tg) * SK + il], KR(s), acc);
        return acc;
    };
    // buffer after b in the rotation
    auto bnext = [](int b) { return PIPE ? (b == NB - 1 ? 0 : b + 1) : (b ^ 1); };
    // one t-tile; `buf` holds its C^ slice.  PIPE: bnext(buf) holds slice
    // tt+1 (its L goes to nx.l) and slice tt+2 is staged into the buffer after
    // that; otherwise slice tt+1 is staged into buf^1.
#if K5_PROF
    uint64_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, plast = 0, psteps = 0;
#endif
    auto body = [&](int64_t tt, int buf, Regs& cx, Regs& nx, bool pf) {
        K5_PT(0);
#if K5_PROF
        ++psteps;
#endif
        const int bL = PIPE ? bnext(buf) : buf;
        const int bS = bnext(bL);
        const int64_t tb = tm_tile_base(tile, phys(tt), ntt);
        const int64_t o = (tb >> 1) + lane;
        // prefetch first; it only needs tile tt+1's dense flag, whose slot
        // arrived with the batch of this tile
        if (pf) {
            const bool dn1 = PRO ? false : ce_is_dense(nx.ce);
            const bool dnp1 = (PRO || !DY) ? false : ce_is_dense(nx.cep);
            stage_load(PIPE ? (tt + 2 < ntt ? tt + 2 : ntt - 1) : tt + 1);
            load(tt + 1, nx);
            if constexpr (DE) {  // both E tiles are part of the regular batch
                load_dense(tt + 1, nx);
                load_dense_p(tt + 1, nx);
            }
            // keep the prefetch ahead of the compute: the scheduler otherwise
            // sinks it next to the stores (less register pressure, no latency
            // hiding)
            __builtin_amdgcn_sched_barrier(0);
            // rare, wave-uniform: tile tt+1 overflowed last time.  Issued after
            // the batch and consumed a step later, so the common path's waits
            // stay exact
            if (!DE && !PRO && dn1) load_dense(tt + 1, nx);
            if (!DE && !PRO && DY && dnp1) load_dense_p(tt + 1, nx);
        }
        K5_PT(1);
        double ev[4], evp[4];
        if constexpr (DE) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    ev[2 * p + q] = cx.ed[p][q];
                    evp[2 * p + q] = cx.edp[p][q];
                }
        } else if (!PRO) {
            const bool dn = ce_decode(cx.ce, lane, img, ev);
#if K5_DNBR
            if (dn) {  // wave-uniform and rare: a scalar branch, not 8 selects
                asm volatile("" ::: "memory");  // keeps it a branch (no if-conversion)
                ev[0] = cx.ed[0][0];
                ev[1] = cx.ed[0][1];
                ev[2] = cx.ed[1][0];
                ev[3] = cx.ed[1][1];
            }
#else
            // (selects, not a branch: a branch would cut the basic block and
            // keep the scheduler from interleaving the decode with the L MFMAs)
            ev[0] = dn ? cx.ed[0][0] : ev[0];
            ev[1] = dn ? cx.ed[0][1] : ev[1];
            ev[2] = dn ? cx.ed[1][0] : ev[2];
            ev[3] = dn ? cx.ed[1][1] : ev[3];
#endif
            if (DY) {
                const bool dp = ce_decode(cx.cep, lane, imgp, evp);
#if K5_DNBR
                if (dp) {
                    asm volatile("" ::: "memory");
                    evp[0] = cx.edp[0][0];
                    evp[1] = cx.edp[0][1];
                    evp[2] = cx.edp[1][0];
                    evp[3] = cx.edp[1][1];
                }
#else
                evp[0] = dp ? cx.edp[0][0] : evp[0];
                evp[1] = dp ? cx.edp[0][1] : evp[1];
                evp[2] = dp ? cx.edp[1][0] : evp[2];
                evp[3] = dp ? cx.edp[1][1] : evp[3];
#endif
            }
            if (pf) load_slot(tt + 2, cx);  // cx.ce (and cx.cep) were consumed above
        }
        K5_PT(2);
        const double* cR = sC[buf];
        // L of t-tile tt+1 (always computed: past the last tile it reads a
        // slice nobody uses, into a register set nobody reads)
        if (PIPE) nx.l = l_mfma(bL);
        double tr[4];
        if (PRO) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const double d = cx.x[0][p][q], yl = cx.x[1][p][q], ov = cx.x[2][p][q];
                    const double tn = (d - ov) + sc.invL * yl;  // :33
                    tr[2 * p + q] = tn;
                }
            }
        } else {
            d4 lacc = {0.0, 0.0, 0.0, 0.0};
            if (PIPE) {
                lacc = cx.l;
            } else {
#if K5_LSPLIT > 1
            // K5_LSPLIT independent accumulation chains over the K-steps, summed
            // in a fixed order (the dependent 16-MFMA chain paces one wave)
            {
                const double* cT = sCT[buf];
                d4 lp[K5_LSPLIT];
#pragma unroll
                for (int c = 0; c < K5_LSPLIT; ++c) lp[c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int s = 0; s < KS; ++s)
                    lp[s % K5_LSPLIT] = mfma4(cT[(4 * s + tg) * SK + il], KR(s), lp[s % K5_LSPLIT]);
                lacc = lp[0];
#pragma unroll
                for (int c = 1; c < K5_LSPLIT; ++c) lacc = lacc + lp[c];
            }
#else
            lacc = l_mfma(buf);
#endif
            }
            K5_PT(3);
            double En[4];
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                d2v YLn2, YOn2;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int r = 2 * p + q;
                    const double d = cx.x[0][p][q], yl = cx.x[1][p][q], e = ev[r];
                    const double L = lacc[r];
#if K5_FUSE
                    // The statements of :41-53 with their multiply-adds fused
                    // and O formed as (R1 + R2)/2 (muL == muO, :16-17,56-57, so
                    // (muL R1 + muO R2)/(muL + muO) is exactly that average);
                    // 18 f64 operations per element instead of 27 (K5 is
                    // bound by the f64 pipe its MFMAs share).
                    // Values agree with the separate-operator forms to
                    // rounding (the parity tolerances of DESIGN.md §2).
                    const double dL = d - L;
                    const double yo = DY ? fma(-sc.muO_prev, e - evp[r], yl) : cx.x[2][p][q];
                    const double R1 = fma(sc.invL, yl, dL);                 // :41
                    const double R2 = fma(-sc.invO, yo, e);                 // :42
                    const double On = (R1 + R2) * 0.5;                      // :43
                    const double R3 = fma(sc.invO, yo, On);                 // :46
                    const double Ev = R3 - fmin(fmax(R3, -sc.thr), sc.thr); // :47
                    const double rL = dL - On;                              // :50
                    const double rO = On - Ev;                              // :51
                    const double YLn = fma(sc.muL, rL, yl);                 // :52
                    const double YOn = fma(sc.muO, rO, yo);                 // :53
                    const double Tn = fma(sc.invL_next, YLn, d - On);       // :33 (k+1)
                    ssL = fma(rL, rL, ssL);
                    ssO = fma(rO, rO, ssO);
#else
                    // DY: Y_O^(k) = Y_L^(k) - muO_k (E^(k) - E^(k-1))  (header)
                    const double yo = DY ? yl - sc.muO_prev * (e - evp[r]) : cx.x[2][p][q];
                    const double R1 = (d - L) + sc.invL * yl;               // :41
                    const double R2 = e - sc.invO * yo;                     // :42
#if K5_FASTDIV
                    // x/den as a reciprocal product with one exact-residual
                    // correction (Markstein: q0 = x*(1/den), r = x - q0*den by
                    // FMA, q = q0 + r*(1/den)); the quotient MATLAB's division
                    // rounds to, in 3 VALU ops instead of the ~11 of the
                    // scaled IEEE sequence (K5 is VALU-issue-bound)
                    const double Onum = sc.muL * R1 + sc.muO * R2;
                    const double q0 = Onum * sc.rden;
                    const double On = fma(fma(-q0, sc.den, Onum), sc.rden, q0);  // :43
#else
                    const double On = (sc.muL * R1 + sc.muO * R2) / sc.den; // :43
#endif
                    const double R3 = On + sc.invO * yo;                    // :46
#if K5_CSIGN == 2
                    // sign(R3).*max(abs(R3)-thr,0) as R3 - clamp(R3,-thr,thr)
                    // (thr >= 0): |R3| > thr gives R3 -/+ thr, the same rounded
                    // difference; otherwise a zero (possibly -0 where MATLAB has
                    // +0); NaN and Inf pass through.  3 VALU ops instead of 10
                    const double Ev = R3 - fmin(fmax(R3, -sc.thr), sc.thr);  // :47
#elif K5_CSIGN
                    // sign(R3).*max(abs(R3)-thr,0) as copysign (thr > 0): equal
                    // values (a zero may come out as -0), NaN kept; 7 VALU ops
                    // instead of 10
                    double Ev = __builtin_copysign(fmax(fabs(R3) - sc.thr, 0.0), R3);  // :47
                    Ev = (R3 != R3) ? R3 : Ev;
#else
                    const double Ev = matlab_sign(R3) * fmax(fabs(R3) - sc.thr, 0.0);  // :47
#endif
                    const double rL = (d - L) - On;                         // :50
                    const double rO = On - Ev;                              // :51
                    const double YLn = yl + sc.muL * rL;                    // :52
                    const double YOn = yo + sc.muO * rO;                    // :53
                    const double Tn = (d - On) + sc.invL_next * YLn;        // :33 (k+1)
#if K5_FASTDIV
                    ssL = fma(rL, rL, ssL);  // norm sums: our own order anyway
                    ssO = fma(rO, rO, ssO);
#else
                    ssL += rL * rL;
                    ssO += rO * rO;
#endif
#endif  // K5_FUSE
                    En[r] = Ev;
                    YLn2[q] = YLn;
                    YOn2[q] = YOn;
                    tr[r] = Tn;
                }
#if K5_BUF
                if (DY) bst(YLn2, rYL, tt, p);
                else
#endif
                st2(YLn2, YL2 + o + 64 * p);
                if (!DY) st2(YOn2, YO2 + o + 64 * p);
            }
            K5_PT(4);
            if constexpr (DE) {  // E^(k+1) over E^(k-1), densely
                st2(d2v{En[0], En[1]}, Eout2 + o);
                st2(d2v{En[2], En[3]}, Eout2 + o + 64);
                ++ndense;
            } else {
#if K5_BUF
                ce_encode_r(En, lane, cs, DY ? rCEp : rCE, (int)(phys(tt) * 1024), Eout2, o, ndense);
#else
                ce_encode(En, lane, cs, CEout, (tb >> 8) * CE_SLOT, Eout2, o, ndense);
#endif
            }
            K5_PT(5);
        }
        // T -> "TX" order (common.h): lane l, slot s holds T(ij = 4s+(l>>4), t = l&15)
        if (K5_EXP & 8) {
#pragma unroll
            for (int p = 0; p < 2; ++p) st2(d2v{tr[2 * p], tr[2 * p + 1]}, T2 + o + 64 * p);
        } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[(tg + 4 * r) * 17 + il] = tr[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            d2v tv;
            tv[0] = ts[il * 17 + 4 * (2 * p) + tg];
            tv[1] = ts[il * 17 + 4 * (2 * p + 1) + tg];
#if K5_BUF
            if (!PRO && DY) bst(tv, rT, tt, p);
            else
#endif
            st2(tv, T2 + o + 64 * p);
        }
        }
        K5_PT(6);
        // W^T(k, ij) += sum_t C^(t,k) T(t, ij): K-step r covers t = t0+4r+(l>>4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (!(K5_EXP & 2)) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                wacc[m] = mfma4(cR[(4 * r + tg) * LDC + 16 * m + il], tr[r], wacc[m]);
            } else {
                for (int m = 0; m < MT; ++m) wacc[m][0] += tr[r];
            }
        }
#if K5_EXP & 48
        {   // timing experiment: extra VALU per t-tile (16: 32 int adds, 32: 16 f64 adds)
            unsigned du = (unsigned)lane;
            double dd = (double)lane;
            if (K5_EXP & 16)
#pragma unroll
                for (int q = 0; q < 32; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(du) : "v"(il));
            if (K5_EXP & 32)
#pragma unroll
                for (int q = 0; q < 16; ++q) asm volatile("v_add_f64 %0, %0, %1" : "+v"(dd) : "v"(dd));
            if (du == 12345u && dd == 1.5) ssL += 1.0;
        }
#endif
        K5_PT(7);
        if (pf) stage_store(bS);  // bS was last read in t-tile tt-1
        if (!(K5_EXP & 4)) __syncthreads();  // C^ buffer `buf` and the T transpose buffer are free again
        // step boundary: the scheduler would otherwise hoist the next step's
        // dense-slot test (which needs this step's loads) above the barrier
        __builtin_amdgcn_sched_barrier(0);
        K5_PT(8);
    };

    Regs xa, xb;
#pragma unroll
    for (int q = 0; q < 3; ++q) xa.x[q][0] = xa.x[q][1] = xb.x[q][0] = xb.x[q][1] = d2v{0.0, 0.0};
    xa.ed[0] = xa.ed[1] = xb.ed[0] = xb.ed[1] = d2v{0.0, 0.0};
    xa.edp[0] = xa.edp[1] = xb.edp[0] = xb.edp[1] = d2v{0.0, 0.0};
    xa.ce = xb.ce = xa.cep = xb.cep = 0.0;
    if (!PRO) {
        load_slot(t0, xa);
        load_slot(t0 + 1, xb);
    }
    load(t0, xa);
    if (DE || (!PRO && ce_is_dense(xa.ce))) load_dense(t0, xa);
    if (DE || (!PRO && DY && ce_is_dense(xa.cep))) load_dense_p(t0, xa);
    stage(t0, 0);
    if (PIPE) stage(t1 - t0 > 1 ? t0 + 1 : t0, 1);
    __syncthreads();
    if (PIPE) xa.l = l_mfma(0);
    xb.l = d4{0.0, 0.0, 0.0, 0.0};
    int64_t tt = t0;
    int b = 0;  // buffer of t-tile tt's C^ slice
    for (; tt + 2 < t1; tt += 2) {
        body(tt, b, xa, xb, true);
        b = bnext(b);
        body(tt + 1, b, xb, xa, true);
        b = bnext(b);
    }
    if (tt + 1 < t1) {
        body(tt, b, xa, xb, true);
        body(tt + 1, bnext(b), xb, xa, false);
    } else {
        body(tt, b, xa, xb, false);
    }
    if (active) {
        // W^T C/D layout: row k = 16m + tg + 4rr, col ij = il; a t-split walk
        // writes its chunk's partial W into set `chunk` (summed by k_w_reduce)
        const int64_t wbase = (tile << 4) + il + chunk * (int64_t)RP * a.plane;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                a.Wk[(int64_t)(16 * m + tg + 4 * rr) * a.plane + wbase] = wacc[m][rr];
    }

#if K5_PROF
    if (!PRO && lane == 0) {
        for (int q = 0; q < 8; ++q) atomicAdd(&g_k5prof[q], (unsigned long long)pacc[q]);
        atomicAdd(&g_k5prof[8], (unsigned long long)psteps);
    }
#endif
    if (!PRO && ndense && lane == 0)  // spread over DENSE_SLOTS counters
        atomicAdd(a.dense_tiles + ((wgi * K5_WAVES + wid) & (DENSE_SLOTS - 1)),
                  (unsigned long long)ndense);
    if (!PRO) {
        // fixed-order block reduction of the residual norms
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            ssL += __shfl_xor(ssL, off);
            ssO += __shfl_xor(ssO, off);
        }
        __shared__ double red[2][K5_WAVES];
        if (lane == 0) {
            red[0][wid] = ssL;
            red[1][wid] = ssO;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double x = 0.0, y = 0.0;
            for (int w = 0; w < K5_WAVES; ++w) {
                x += red[0][w];
                y += red[1][w];
            }
            a.partial[2 * wgi] = x;
            a.partial[2 * wgi + 1] = y;
        }
    }
    WT_END(g_wt_k5, PRO ? -1 : bid * K5_WAVES + (threadIdx.x >> 6));
}

int k5_grid(const Geom& g) { return (int)cdiv(g.tiles, K5_WAVES); }

// t-split of the fp64 K5 walk: a problem with few ij-tiles (the sensor shape
// 54x4x1152: 16 ij-tiles, 4 workgroups walking 72 t-tiles each) leaves the GPU
// almost idle, so the walk is cut into chunks of >= 8 t-tiles until there are
// about 256 workgroups; each chunk's W is a partial sum (k_w_reduce).
int k5_tsplit(const Geom& g) {
    if (g.RP > 64) return 1;
    const int64_t wg = cdiv(g.tiles, K5_WAVES);
    const int64_t smax = g.ntt / 8 > 1 ? g.ntt / 8 : 1;  // chunks of >= 8 t-tiles
    if (const char* e = std::getenv("TRITD_K5_TSPLIT")) {  // A/B override
        const int64_t f = std::atoll(e);
        return (int)(f < 1 ? 1 : (f > g.ntt ? g.ntt : f));
    }
    if (wg < 256) {  // too few ij-tiles to fill the GPU: ~256 workgroups
        const int64_t s = std::min(cdiv(256, wg), smax);
        return (int)(s < 1 ? 1 : s);
    }
    // (Splitting to fill the rounds of 512 workgroups, e.g. config 3's 1 200
    // = 2.34 rounds, measured slower: K5 0.250 -> 0.261 ms with 2 chunks; the
    // walks are HBM-bound, so a thin last round still streams at full rate.)
    return 1;
}

// Wk (set 0) = sum of the t-split partial sets, in chunk order
__global__ __launch_bounds__(256) void k_w_reduce(double* Wk, int64_t stride, int sets,
                                                  const int* stop) {
    if (*stop) return;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < stride;
         e += (int64_t)gridDim.x * 256) {
        double s = Wk[e];
        for (int c = 1; c < sets; ++c) s += Wk[c * stride + e];
        Wk[e] = s;
    }
}

#if K5_PROF
}  // namespace tritd
// timing experiments only (tools/k5_prof.py): read and clear the phase clocks
extern "C" int tritd_k5prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(tritd::g_k5prof), 16 * sizeof(unsigned long long)) !=
        hipSuccess)
        return 1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(tritd::g_k5prof), z, sizeof z) == hipSuccess ? 0 : 1;
}
namespace tritd {
#endif

void launch_k5(const Geom& g, const K5Args& a, bool prologue, bool dy, hipStream_t st, bool dense_e) {
    if (a.side.on && (prologue || g.RP > 64)) throw Error(TRITD_ERR_ARG, "K5 side solve: RP <= 64 only");
    if (dense_e && (prologue || !dy || g.RP > 64))
        throw Error(TRITD_ERR_ARG, "K5 dense-E mode: derived-Y_O update, RP <= 64");
    K5Args b = a;  // (the macro below launches with `b`)
    b.tsplit = k5_tsplit(g);
    const dim3 grid(k5_grid(g) * b.tsplit + (a.side.on ? 1 : 0)), block(64 * K5_WAVES);
#define K5_CASE(RPV)                                                                       \
    case RPV:                                                                              \
        if (prologue)                                                                      \
            hipLaunchKernelGGL((k5_fused<RPV, true, false>), grid, block, 0, st, b);       \
        else if (dy && dense_e && RPV <= 64)                                               \
            hipLaunchKernelGGL((k5_fused<RPV, false, true, (RPV <= 64)>), grid, block, 0, st, b); \
        else if (dy)                                                                       \
            hipLaunchKernelGGL((k5_fused<RPV, false, true>), grid, block, 0, st, b);       \
        else                                                                               \
            hipLaunchKernelGGL((k5_fused<RPV, false, false>), grid, block, 0, st, b);      \
        break;
    switch (g.RP) {
        K5_CASE(16)
        K5_CASE(32)
        K5_CASE(48)
        K5_CASE(64)
        K5_CASE(128)  // r = 9..16 (fp64): one wave per SIMD, 146 KB of LDS at 256
        K5_CASE(256)
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by K5");
    }
#undef K5_CASE
    TRITD_CHECK_LAUNCH();
    if (b.tsplit > 1) {
        const int64_t stride = (int64_t)g.RP * g.plane;
        hipLaunchKernelGGL(k_w_reduce, dim3((unsigned)std::min<int64_t>(cdiv(stride, 256), 2048)),
                           dim3(256), 0, st, b.Wk, stride, b.tsplit, b.stop);
        TRITD_CHECK_LAUNCH();
    }
}

// Sum n (x, y) pairs in a fixed order: per-thread strided sums, then a
// fixed tree.  One block.
__global__ __launch_bounds__(256) void k_reduce_pairs(const double* __restrict__ p, int n,
                                                      double* out, const int* stop) {
    if (stop && *stop) return;
    __shared__ double sx[256], sy[256];
    double x = 0.0, y = 0.0;
#pragma unroll 8  // loads batched; the sums keep their sequential order
    for (int b = threadIdx.x; b < n; b += 256) {
        x += p[2 * b];
        y += p[2 * b + 1];
    }
    sx[threadIdx.x] = x;
    sy[threadIdx.x] = y;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sx[threadIdx.x] += sx[threadIdx.x + w];
            sy[threadIdx.x] += sy[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = sx[0];
        out[1] = sy[0];
    }
}

void launch_reduce_pairs(const double* partial, int n, double* out, const int* stop,
                         hipStream_t st) {
    hipLaunchKernelGGL(k_reduce_pairs, dim3(1), dim3(256), 0, st, partial, n, out, stop);
    TRITD_CHECK_LAUNCH();
}

// ctrl[0] = stop flag, ctrl[1] = iterations completed (k of :68)
__device__ __forceinline__ void finish_body(const double* ss, double normD, int k, double tol,
                                            double* errHist, double* errL, double* errO, int* ctrl,
                                            int single) {
    double eL = sqrt(ss[0]) / normD;  // norm(resL(:))/normD
    double eO = sqrt(ss[1]) / normD;  // norm(resO(:))/normD
    double e = eL + eO;               // :59
    if (single) {  // single residuals: single norms, single quotients and sum
        const float fL = (float)sqrt(ss[0]) / (float)normD;
        const float fO = (float)sqrt(ss[1]) / (float)normD;
        eL = fL;
        eO = fO;
        e = (double)(fL + fO);
    }
    errHist[k - 1] = e;
    errL[k - 1] = eL;
    errO[k - 1] = eO;
    ctrl[1] = k;
    if (k > 1 && fabs(e - errHist[k - 2]) < tol * errHist[k - 2]) ctrl[0] = 1;  // :63
}

__global__ void k_finish(const double* ss, double normD, int k, double tol, double* errHist,
                         double* errL, double* errO, int* ctrl, int single) {
    if (ctrl[0]) return;
    finish_body(ss, normD, k, tol, errHist, errL, errO, ctrl, single);
}

// clear: zero the pairs after reading them (each thread clears the pairs it
// read).  The sharded schedule's norm partials live in red1_'s tail, sized to
// the largest shard's K5 grid; a rank with fewer workgroups leaves the slots
// past its own at zero, and the all-reduce writes sums into all of them.
__global__ __launch_bounds__(256) void k_reduce_finish(double* __restrict__ p, int n,
                                                       double normD, int k, double tol,
                                                       double* errHist, double* errL, double* errO,
                                                       int* ctrl, int single, int clear) {
    if (ctrl[0]) return;
    __shared__ double sx[256], sy[256];
    double x = 0.0, y = 0.0;
#pragma unroll 8  // loads batched; the sums keep their sequential order
    for (int b = threadIdx.x; b < n; b += 256) {
        x += p[2 * b];
        y += p[2 * b + 1];
    }
    if (clear)
        for (int b = threadIdx.x; b < n; b += 256) {
            p[2 * b] = 0.0;
            p[2 * b + 1] = 0.0;
        }
    sx[threadIdx.x] = x;
    sy[threadIdx.x] = y;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sx[threadIdx.x] += sx[threadIdx.x + w];
            sy[threadIdx.x] += sy[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double ss[2] = {sx[0], sy[0]};
        finish_body(ss, normD, k, tol, errHist, errL, errO, ctrl, single);
    }
}

void launch_reduce_finish(double* partial, int n, double normD, int k, double tol,
                          double* errHist, double* errL, double* errO, int* ctrl, bool single,
                          hipStream_t st, bool clear) {
    hipLaunchKernelGGL(k_reduce_finish, dim3(1), dim3(256), 0, st, partial, n, normD, k, tol,
                       errHist, errL, errO, ctrl, (int)single, (int)clear);
    TRITD_CHECK_LAUNCH();
}

void launch_finish(const double* ss, double normD, int k, double tol, double* errHist, double* errL,
                   double* errO, int* ctrl, bool single, hipStream_t st) {
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(1), 0, st, ss, normD, k, tol, errHist, errL, errO,
                       ctrl, (int)single);
    TRITD_CHECK_LAUNCH();
}

// O_k = (D + (1/muL_{k+1}) Y_L) - T_{k+1}: D, Y_L, O in tile-major order,
// T in the TX order of the same tile (common.h)
__global__ __launch_bounds__(256) void k_o_fixup(const double* __restrict__ D,
                                                 const double* __restrict__ YL,
                                                 const double* __restrict__ T, double invL_next,
                                                 double* __restrict__ O, int64_t Np) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < Np; e += (int64_t)gridDim.x * 256) {
        const int w = (int)(e & 255);
        const int p = w >> 7, l = (w & 127) >> 1, q = w & 1;
        const int r = 2 * p + q;
        const int il = l & 15, tl = (l >> 4) + 4 * r;  // element of this TM slot
        const int s = il >> 2, lx = ((il & 3) << 4) | tl;  // its TX slot
        const int64_t tx = (e & ~(int64_t)255) + ((s >> 1) << 7) + (lx << 1) + (s & 1);
        O[e] = (D[e] + invL_next * YL[e]) - T[tx];
    }
}

void launch_o_fixup(const Geom& g, const double* D, const double* YL, const double* T,
                    double invL_next, double* O, hipStream_t st) {
    int64_t b = cdiv(g.Ntm, 256);
    if (b > 16384) b = 16384;
    hipLaunchKernelGGL(k_o_fixup, dim3((unsigned)b), dim3(256), 0, st, D, YL, T, invL_next, O, g.Ntm);
    TRITD_CHECK_LAUNCH();
}

// Placement probe: K5's HBM pattern (read D, Y_L, Y_O (not with dy) and the
// tile's 256 B compact-E slot; write Y_L, Y_O (not with dy) in place, T and
// the slot; one wave per ij-tile walking its t-tiles, prefetched) without the
// arithmetic.  K5 is HBM-bound and its bandwidth depends on where the pool
// landed physically; the session times candidate pools with this and keeps
// the fastest.  Contents are overwritten with garbage.
template <bool DY>
__global__ __launch_bounds__(256) void k_pool_probe(double* D, double* YL, double* YO, double* T,
                                                    double* CE, int64_t tiles4, int64_t ntt) {
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= tiles4) return;
    d2v* P[4] = {reinterpret_cast<d2v*>(D), reinterpret_cast<d2v*>(YL), reinterpret_cast<d2v*>(YO),
                 reinterpret_cast<d2v*>(T)};
    auto tb = [&](int64_t tt) { return tm_tile_base(tile, tt, ntt); };
    struct R {
        d2v x[3][2];
        double ce;
    };
    R xa, xb;
    auto load = [&](int64_t tt, R& nx) {
        const int64_t o = (tb(tt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int f = 0; f < (DY ? 2 : 3); ++f) nx.x[f][p] = P[f][o + 64 * p];
        nx.ce = CE[(tb(tt) >> 8) * CE_SLOT + (lane & 31)];
    };
    auto body = [&](int64_t tt, R& c, R& n, bool pf) {
        if (pf) {
            load(tt + 1, n);
            __builtin_amdgcn_sched_barrier(0);
        }
        const int64_t o = (tb(tt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            if (DY) {
                P[1][o + 64 * p] = c.x[0][p] + c.x[1][p];
                P[3][o + 64 * p] = c.x[0][p] - c.x[1][p];
            } else {
                P[1][o + 64 * p] = c.x[0][p] + c.x[1][p];
                P[2][o + 64 * p] = c.x[2][p] - c.x[1][p];
                P[3][o + 64 * p] = c.x[0][p] - c.x[2][p];
            }
        }
        CE[(tb(tt) >> 8) * CE_SLOT + (lane & 31)] = c.ce + 1.0;
    };
    load(0, xa);
    int64_t tt = 0;
    for (; tt + 2 < ntt; tt += 2) {
        body(tt, xa, xb, true);
        body(tt + 1, xb, xa, true);
    }
    if (tt + 1 < ntt) {
        body(tt, xa, xb, true);
        body(tt + 1, xb, xa, false);
    } else {
        body(tt, xa, xb, false);
    }
}

void launch_pool_probe(const Geom& g, double* D, double* YL, double* YO, double* T, double* CE,
                       bool dy, hipStream_t st) {
    if (dy)
        hipLaunchKernelGGL(k_pool_probe<true>, dim3((unsigned)(g.tiles4 / 4)), dim3(256), 0, st, D,
                           YL, YO, T, CE, g.tiles4, g.ntt);
    else
        hipLaunchKernelGGL(k_pool_probe<false>, dim3((unsigned)(g.tiles4 / 4)), dim3(256), 0, st, D,
                           YL, YO, T, CE, g.tiles4, g.ntt);
    TRITD_CHECK_LAUNCH();
}

// Compact E -> dense E (TM) for every tile that is not already dense: one
// wave per tile ordinal (common.h: CE).
__global__ __launch_bounds__(256) void k_ce_expand(const double* __restrict__ CE, double* E,
                                                   int64_t ntiles) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= ntiles) return;
    __shared__ double cimg[4][CE_IMG];
    double* img = cimg[threadIdx.x >> 6];
    for (int e = lane; e < CE_IMG; e += 64) img[e] = 0.0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const double sv = CE[b * CE_SLOT + (lane & 31)];
    double e[4];
    if (ce_decode(sv, lane, img, e)) return;  // dense tile: E already holds it
    d2v* E2 = reinterpret_cast<d2v*>(E) + b * 128 + lane;
    E2[0] = d2v{e[0], e[1]};
    E2[64] = d2v{e[2], e[3]};
}

void launch_ce_expand(const Geom& g, const double* CE, double* E, hipStream_t st) {
    const int64_t ntiles = g.Ntm / 256;
    hipLaunchKernelGGL(k_ce_expand, dim3((unsigned)cdiv(ntiles, 4)), dim3(256), 0, st, CE, E, ntiles);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
