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
// in one pass: reads D and Y_L and writes Y_L and T (4 dense N-streams),
// reads E^(k), E^(k-1) and writes E^(k+1) in their compact form (one 256 B
// slot per 2 KB tile, common.h; dense only for overflowed tiles), plus W
// (N*R/n3 elements).  O is never read inside the loop (E, not O, feeds :42),
// so it is not stored: T_{k+1} = (D - O_k) + Y_L/muL_{k+1} determines it and
// k_o_fixup rebuilds O_k = (D + Y_L/muL_{k+1}) - T_{k+1} when the caller asks
// for it (relative error ~1e-16).
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
// Derived Y_O: with muL == muO (both are opts.mu, :16-17, and follow one
// schedule, :56-57), :43 gives 2 O = (D - L) + E^(k-1) + (Y_L - Y_O)/mu,
// hence from :51-53
//   Y_L^(k) - Y_O^(k) = (Y_L - Y_O) + mu (D - L - 2 O + E^(k)) = mu_k (E^(k) - E^(k-1))
// exactly, for every k (Y_L^(0) = Y_O^(0) = 0).  So Y_O is never stored: the
// K5 of iteration k+1 reads Y_L^(k) and the compact E^(k), E^(k-1) (256 B per
// tile each) and forms Y_O^(k) = Y_L^(k) - mu_k (E^(k) - E^(k-1)).  The
// rebuilt Y_O differs from MATLAB's by rounding only (checked against the
// restatement on every golden case: L, O, E within 1e-11, same k;
// tests/test_gpu_parity.py holds the GPU to 1e-9).
//
// Parity contract of the elementwise chain.  The file is compiled with
// -ffp-contract=off, so the compiler fuses nothing on its own.  The chain
// requests FMAs explicitly in the statements of :41-53 and forms O as
// (R1 + R2)/2 (exact for muL == muO): its values agree with MATLAB's
// separate operators to rounding, not bit for bit, and the tests hold it to
// the tolerances of DESIGN.md §2 (L, O, E 1e-9; errHist 1e-8 relative; the
// same k, including a near-tolerance stop golden).  The norm sums of :59 use
// FMAs too: their summation order is this kernel's own (per lane, then a
// fixed-order tree), never MATLAB's.
#include "finish.h"
#include "kernels.h"
#include "sweep.h"
#include "wtrace.h"

namespace tritd {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

// Waves per workgroup: exactly one group of 4 ij-tiles (common.h: the TM
// layout interleaves groups of 4 and pads tiles4 to a multiple of 4, so a
// wider workgroup would stream past the allocation; 8 waves measured no
// faster).
static constexpr int K5_WAVES = 4;
// Waves per SIMD at RP <= 64 (VGPR + AGPR <= 256).  One wave per SIMD: 1.243
// vs 0.998 ms (round 2); three need <= 168 VGPRs and spill.
#ifndef TRITD_K5_WPE
#define TRITD_K5_WPE 2
#endif
static constexpr int K5_WPE = TRITD_K5_WPE;
// Nontemporal hint (buffer aux bit 1) on the streamed tensors, loads and
// stores: round 2 interleaved A/B, nt stores -1.5 % iteration, nt loads a
// further -0.9 % (M1 then finds W still in the Infinity Cache).
static constexpr int K5_NT_AUX = 2;
// 1: the data of every wide store is held live past a later point (below,
// DESIGN.md §4.2).  0 exists only so that tests/test_isa_store_war.py can
// build the kernel without the keeps and check that its scan catches them.
#ifndef TRITD_STORE_KEEP
#define TRITD_STORE_KEEP 1
#endif

#if TRITD_WTRACE
WT_DECL(g_wt_k5)
#endif

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// --- compact E (common.h: CE) -------------------------------------------
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
// Store this lane's 4 elements of E (register order) as the tile's slot
// (buffer rs at scalar offset soff), or densely into E2 at d2v offset o when
// they do not fit.  cs: the wave's 96-double LDS scratch (slot image + a junk
// area for the zeros).  Branch-free: a branch here makes the compiler's
// vmcnt waits drain the prefetch.
__device__ __forceinline__ void ce_encode(const double (&En)[4], int lane, double* cs,
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
        // junk area).  The wave-uniform mask itself is the lane condition
        // (inverse ballot: one select, no shift/and/compare).
        const bool bit = !dense && __builtin_amdgcn_inverse_ballot_w64(nz[w]);
        // One select for both writes: a lane with no value writes word 32 +
        // lane and byte CE_IDX_BYTE + 32 + lane (word 31 and up: the count
        // word, written after this loop in the same wave's LDS order, and the
        // junk area); mbcnt takes `pre` as its addend.  (Round 6: bitwise the
        // same slots, K5 0.915 -> 0.908 ms, profiles/round6/ce_encode_ab.txt.)
        const int at = (int)__builtin_amdgcn_mbcnt_hi(
            (uint32_t)(nz[w] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nz[w], (uint32_t)pre));
        const int sel = bit ? at : 32 + lane;
        cs[sel] = En[w];
        cb[CE_IDX_BYTE + sel] = (unsigned char)(64 * w + lane);
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

// K5, the fused update of iteration k (PRO = false) or the prologue that
// forms T of iteration 1 and W from it (PRO = true).
//
// Derived Y_O: Y_O^(k) is rebuilt from Y_L^(k) and the compact E^(k) (CE/E)
// and E^(k-1) (CEp/Ep); E^(k+1) is written over E^(k-1).
// DE (dense-E mode): E^(k), E^(k-1) and E^(k+1) live densely in the
// tile-major E buffers for every tile — no compact slots are read, decoded,
// encoded or written.  The session switches to it once E has turned dense
// (video-like data: every tile overflows its slot and the compact form only
// adds the slot traffic and the decode/encode work; solver.cpp run()).
template <int RP, bool PRO, bool DE = false>
__global__ __launch_bounds__(64 * K5_WAVES) __attribute__((amdgpu_waves_per_eu(RP >= 128 ? 1 : K5_WPE, K5_WPE)))
void k5_fused(K5Args a) {
    static_assert(!DE || !PRO, "k5_fused: dense-E mode is an update, not the prologue");
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
    // 4 ij-tiles.  (Round 6: one workgroup walking 2 or 4 such units in turn,
    // bitwise the same results, measured K5 0.933 / 0.934 vs 0.919 ms —
    // profiles/round6/k5_ab/ab_k5_units_per_workgroup_dropped.txt: the
    // workgroup turnover is not where the per-walk fixed cost goes.)
    // (index arithmetic in 32 bits: every count here is far below 2^32, and
    // a 64-bit division is ~100 scalar instructions of every workgroup's start)
    const uint32_t wgi = blockIdx.x - (uint32_t)side;
    const uint32_t ngrp = (uint32_t)((a.tiles + K5_WAVES - 1) / K5_WAVES);
    const uint32_t chunk = wgi / ngrp;
    const uint32_t bid = wgi - chunk * ngrp;  // this workgroup's group of ij-tiles
    WT_BEGIN();
    constexpr int KS = RP / 4;   // MFMA K-steps for L
    constexpr int MT = RP / 16;  // k-tiles of W
    const int lane = threadIdx.x & 63;
    // wave-uniform in SGPRs: every tile base below becomes scalar address math
    // (K5 is VALU-issue-bound)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int il = lane & 15;
    const int tg = lane >> 4;
    const int64_t tile = (int64_t)bid * K5_WAVES + wid;
    const bool active = tile < a.tiles;
    const uint32_t qper = (uint32_t)(a.n1p >> 4);
    const int64_t j = active ? (uint32_t)tile / qper : 0;
    const int64_t i = active ? ((tile - j * qper) << 4) + il : 0;
    const int64_t ntt = a.ntt;
    const int64_t t0 = chunk * (uint32_t)ntt / (uint32_t)a.tsplit;  // this chunk's t-tiles
    const int64_t t1 = (chunk + 1) * (uint32_t)ntt / (uint32_t)a.tsplit;

    // C^ rows of one t-tile, staged once per workgroup in ONE layout read by
    // both MFMA chains: element (t, k) at t*LDP + 2*(t>>1) + k, LDP = 16 mod
    // 32 doubles.  ds_read_b64 banks (a/4) mod 64 per 32-lane half
    // (MI355X_MICROARCH.md §LDS): the L operand (t = l&15, k = 4s+(l>>4)) and
    // the W operand (t = 4r+(l>>4), k = 16m+(l&15)) both touch 32 distinct
    // bank pairs per half, and the staging ds_write_b128 8 distinct 16-B
    // slots per 8-lane group; every operand address is a per-lane base plus
    // an immediate.  Four buffers, staged SD = 2 t-tiles ahead, so a barrier
    // closes every second t-tile only (the buffer a step stages was read two
    // steps earlier, and is read two steps later).  Round 4, against round 3's
    // two layouts ([t][k] and [k][t] copies, double-buffered, a barrier per
    // t-tile): K5 0.960 -> 0.924 ms, iteration 1.366 -> 1.330 ms (6
    // interleaved pairs, profiles/round4/ab_k5_one_layout.txt).
    constexpr int LDP = ((RP + 31) / 32) * 32 + 16;
    constexpr int SLICE = 16 * LDP + 16;
#ifndef TRITD_K5_NBUF  // A/B builds only (round 6: the 3-waves-per-SIMD study)
#define TRITD_K5_NBUF 4
#endif
#ifndef TRITD_K5_PF
#define TRITD_K5_PF 1
#endif
    constexpr int NBUF = TRITD_K5_NBUF, SD = NBUF / 2;
    constexpr bool PF = TRITD_K5_PF != 0;  // tile tt+1 prefetched into the second register set
    __shared__ __attribute__((aligned(16))) double sCS[NBUF][SLICE];
    auto slice_buf = [](int64_t s) { return (int)(s & (NBUF - 1)); };
    // per-wave 16x16 transpose buffer for T (stored in the M3 B-operand order)
    __shared__ double tsm[K5_WAVES][16 * 17];
    double* ts = tsm[wid];
    // Staging is split so that its global loads are issued before the tile
    // prefetch and its LDS writes come after this t-tile's compute: vmcnt is
    // in-order, so a wait on a load issued after the prefetch would also wait
    // for the prefetch (measured: the prefetch was serialized every t-tile).
    constexpr int SP = 16 * RP / 2;                 // (v0,v1) pairs per slice
    constexpr int NS = (SP + 64 * K5_WAVES - 1) / (64 * K5_WAVES);
    d2v sv[NS];
    // C^ slices through one descriptor: slice tt at a scalar offset
    const __amdgpu_buffer_rsrc_t rCh = wave_rsrc(a.Ch, (int)(a.n3p * RP * 8));
    auto stage_load_to = [&](int64_t tt, d2v (&dst)[NS]) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5_WAVES;
            if (SP % (64 * K5_WAVES) == 0 || e < SP)
                dst[q] = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rCh, 16 * e, (int)(tt * 16 * RP * 8), 0));
        }
    };
    auto stage_store_from = [&](int buf, const d2v (&src)[NS]) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5_WAVES;
            if (SP % (64 * K5_WAVES) == 0 || e < SP) {
                const int row = (2 * e) / RP, k = (2 * e) % RP;
                *reinterpret_cast<d2v*>(&sCS[buf][row * LDP + 2 * (row >> 1) + k]) = src[q];
            }
        }
    };
    auto stage_load = [&](int64_t tt) { stage_load_to(tt, sv); };
    auto stage_store = [&](int buf) { stage_store_from(buf, sv); };
    // operand reads: L (t = il, k = 4s+tg) and W (t = 4r+tg, k = 16m+il)
    const int offL = il * LDP + 2 * (il >> 1) + tg;
    const int offW = tg * LDP + 2 * (tg >> 1) + il;
    auto opL = [&](int buf, int s) { return sCS[buf][offL + 4 * s]; };
    auto opW = [&](int buf, int r, int m) { return sCS[buf][offW + r * (4 * LDP + 4) + 16 * m]; };

    // the Khatri-Rao operand of this ij-tile: KR(ij, 4s+tg) (CP or Qi,
    // kernels.h), gathered in the prologue below
    double kr[KS];
    d4 wacc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) wacc[m] = d4{0.0, 0.0, 0.0, 0.0};

    double ssL = 0.0, ssO = 0.0;
    unsigned ndense = 0;  // E tiles of this wave stored densely (wave-uniform)
    const IterScalars sc = a.s;
    const d2v* E2 = reinterpret_cast<const d2v*>(a.E);
    d2v* Ep2 = reinterpret_cast<d2v*>(a.Ep);  // E^(k-1) dense tiles, E^(k+1) destination

    // Two register sets: x[0] = D, x[1] = Y_L (PRO: x[2] = O), ce / cep the
    // lane's word of the compact slots of E^(k) / E^(k-1) (DE: ed / edp the
    // dense tiles).  The t-walk is unrolled by two so that the sets alternate
    // by name: a copy cur = next would make the compiler wait for the
    // prefetch at the copy.  Slots are loaded two tiles ahead.  Nothing
    // depends on `active` (a wave past the last tile streams the zero-filled
    // group padding), so the compiler's in-order vmcnt waits stay exact.
    struct Regs {
        d2v x[PRO ? 3 : 2][2];
        d2v ed[2];
        double ce;
        d2v edp[2];
        double cep;
    };
    __shared__ double csm[K5_WAVES][96];
    double* cs = csm[wid];
    // compact-E decode images (ce_decode), zero between uses: one per slot
    // stream (E^(k), E^(k-1)) where the LDS allows, else shared
    constexpr int NIMG = (DE || PRO) ? 0 : (RP <= 64 ? 2 : 1);
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
        sizeof(double) * (NBUF * SLICE + K5_WAVES * 16 * 17 +
                          K5_WAVES * 96 + (NIMG > 0 ? K5_WAVES * NIMG : 1) * CE_IMG + 2 * K5_WAVES);
    static_assert(LDS_BYTES <= 160 * 1024, "k5_fused: LDS over the 160 KiB of a CU");
    // D, Y_L, T (PRO: O) through buffer descriptors based at this wave's first
    // tile: the t-tile offset is a scalar (soffset), the lane offset a
    // constant VGPR, so the streams need no per-step 64-bit address VALU
    // (tm_tile_base = wave base + tt * 1024 doubles)
    const int64_t wbase = tm_tile_base(tile, 0, ntt);
    const int wbytes = (int)(ntt * 8192);
    const __amdgpu_buffer_rsrc_t rD = wave_rsrc(a.D + wbase, wbytes);
    const __amdgpu_buffer_rsrc_t rYL = wave_rsrc(a.YL + wbase, wbytes);
    const __amdgpu_buffer_rsrc_t rT = wave_rsrc(a.T + wbase, wbytes);
    const __amdgpu_buffer_rsrc_t rO = wave_rsrc(PRO ? a.O + wbase : a.D, PRO ? wbytes : 0);
    const int vlane = lane * 16;
    auto bld = [&](__amdgpu_buffer_rsrc_t r, int64_t tt, int p) {
        return __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(
                                            r, vlane + 1024 * p, (int)(tt * 8192), K5_NT_AUX));
    };
    auto bst = [&](d2v v, __amdgpu_buffer_rsrc_t r, int64_t tt, int p) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), r, vlane + 1024 * p,
                                               (int)(tt * 8192), K5_NT_AUX);
    };
    auto load = [&](int64_t tt, Regs& nx) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            nx.x[0][p] = bld(rD, tt, p);
            nx.x[1][p] = bld(rYL, tt, p);
            if constexpr (PRO) nx.x[PRO ? 2 : 0][p] = bld(rO, tt, p);
        }
    };
    auto load_dense = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tm_tile_base(tile, tt, ntt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p) nx.ed[p] = E2[o + 64 * p];
    };
    auto load_dense_p = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tm_tile_base(tile, tt, ntt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p) nx.edp[p] = Ep2[o + 64 * p];
    };
    // compact-E slots: 4 slots (1 KB) per t-tile from the wave's first one
    const int64_t wslot = (tm_tile_base(tile, 0, ntt) >> 8) * CE_SLOT;
    const __amdgpu_buffer_rsrc_t rCE = wave_rsrc(a.CE + wslot, (int)(ntt * 1024));
    const __amdgpu_buffer_rsrc_t rCEp = wave_rsrc(a.CEp + wslot, (int)(ntt * 1024));
    const int vslot = (lane & 31) * 8;
    auto load_slot = [&](int64_t tt, Regs& rx) {
        if constexpr (DE || PRO) return;
        const int so = (int)((tt < ntt ? tt : ntt - 1) * 1024);  // clamped: no branch
        rx.ce = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rCE, vslot, so, 0));
        rx.cep = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rCEp, vslot, so, 0));
    };

    // one t-tile: cx holds its data, `buf` its C^ slice; if `pf`, tile tt+1 is
    // prefetched into nx and its C^ slice staged into buf^1
    // rare, wave-uniform: an overflowed tile's values are in the dense buffer,
    // loaded when met (a wait on this wave's outstanding loads).  Round 4: the
    // same speed as prefetching them into two more register sets one step
    // ahead (K5 0.949 vs 0.949 ms, 6 interleaved pairs), without that form's
    // 11 spilled VGPRs.
    auto dense_fix = [&](int64_t tt, bool dn, bool dp, double (&ev)[4], double (&evp)[4]) {
        if (dn || dp) {
            const int64_t od = (tm_tile_base(tile, tt, ntt) >> 1) + lane;
            const d2v a0 = E2[od], a1 = E2[od + 64], b0 = Ep2[od], b1 = Ep2[od + 64];
            ev[0] = dn ? a0[0] : ev[0];
            ev[1] = dn ? a0[1] : ev[1];
            ev[2] = dn ? a1[0] : ev[2];
            ev[3] = dn ? a1[1] : ev[3];
            evp[0] = dp ? b0[0] : evp[0];
            evp[1] = dp ? b0[1] : evp[1];
            evp[2] = dp ? b1[0] : evp[2];
            evp[3] = dp ? b1[1] : evp[3];
        }
    };
    // one t-tile: cx holds its data; pf: tile tt+1 is loaded into nx; ps: the
    // C^ slice SD t-tiles ahead is staged; bar: the step ends at a barrier
    auto body = [&](int64_t tt, int buf, Regs& cx, Regs& nx, bool pf, bool ps, bool bar) {
        const int64_t o = (tm_tile_base(tile, tt, ntt) >> 1) + lane;
        // prefetch first
        if (ps) stage_load(tt + SD);
        if (!PF) {  // (A/B: no register prefetch; other waves cover the latency)
            load(tt, cx);
            if constexpr (DE) {
                load_dense(tt, cx);
                load_dense_p(tt, cx);
            }
        }
        if (pf && PF) {
            load(tt + 1, nx);
            if constexpr (DE) {  // both E tiles are part of the regular batch
                load_dense(tt + 1, nx);
                load_dense_p(tt + 1, nx);
            }
        }
        // keep the prefetch ahead of the compute: the scheduler otherwise
        // sinks it next to the stores (less register pressure, no latency
        // hiding)
        __builtin_amdgcn_sched_barrier(0);
        double ev[4], evp[4];
        bool dn = false, dp = false;
        if constexpr (DE) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    ev[2 * p + q] = cx.ed[p][q];
                    evp[2 * p + q] = cx.edp[p][q];
                }
        } else if (!PRO) {
            // (selects, not a branch, for a dense tile: a branch would cut the
            // basic block and keep the scheduler from interleaving the decode
            // with the L MFMAs)
            dn = ce_decode(cx.ce, lane, img, ev);
            dp = ce_decode(cx.cep, lane, imgp, evp);
            dense_fix(tt, dn, dp, ev, evp);
            if (pf) load_slot(tt + 2, cx);  // cx.ce and cx.cep were consumed above
        }
        double tr[4], En[4];
        // The data of this step's wide stores (Y_L, E, T) is held live past
        // a later point (the asm statements below), so the register
        // allocator cannot rewrite those registers right behind the store.
        // Round 4, measured: without it the dense-E form wrote a wrong first
        // 8-byte word in lanes 12-15 of each 16 of a Y_L store now and then
        // (tens of elements per launch at config 3's shape, not
        // reproducible run to run), where the compiler placed a 64-bit VALU
        // write of the data registers 3-4 instructions after a
        // buffer_store_dwordx4 — the signature tools/store_hazard.hip shows
        // for a rewrite with no wait state.  Costs no time (K5 0.934 vs
        // 0.933 ms, profiles/round4/ab_k5_keep.txt).
        d2v keep[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) keep[q] = d2v{0.0, 0.0};
        if constexpr (PRO) {
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const double d = cx.x[0][p][q], yl = cx.x[1][p][q], ov = cx.x[PRO ? 2 : 0][p][q];
                    tr[2 * p + q] = (d - ov) + sc.invL * yl;  // :33
                }
        } else {
            // L^T(t, ij) of this t-tile: KS dependent MFMAs
            d4 lacc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < KS; ++s) lacc = mfma4(opL(buf, s), kr[s], lacc);
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                d2v YLn2;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int r = 2 * p + q;
                    const double d = cx.x[0][p][q], yl = cx.x[1][p][q], e = ev[r];
                    const double L = lacc[r];
                    // The statements of :41-53 with their multiply-adds fused
                    // and O formed as (R1 + R2)/2 (muL == muO, :16-17,56-57, so
                    // (muL R1 + muO R2)/(muL + muO) is exactly that average);
                    // 17 f64 operations per element instead of 27 (K5 is
                    // bound by the SIMD issue its MFMAs share).
                    // Values agree with MATLAB's separate operators to
                    // rounding (the parity tolerances of DESIGN.md §2).
                    // Y_O^(k) = Y_L^(k) - muO_k (E^(k) - E^(k-1))  (derived Y_O)
                    // With Y_O = Y_L - muO_prev dE (dE = E^(k) - E^(k-1)) and
                    // invL = invO: R1 + R2 = (D - L) + invL Y_L + E - invO Y_O
                    // = dL + E + cprev dE (cprev = invO muO_prev) and R3 = On +
                    // invO Y_O = On + invO Y_L - cprev dE — 7 f64 operations
                    // for :41-46 instead of 8 through Y_O (round 6: K5 0.922 ->
                    // 0.915 ms, profiles/round6/k5_chain_dE_ab.txt).  (Starting
                    // the L MFMA chain from D with -KR, so that it leaves D - L,
                    // measured slower: 0.912 -> 0.923 ms, k5_dL_mfma_dropped.txt.)
                    const double dL = d - L;
                    const double dE = e - evp[r];
                    const double On = (dL + fma(sc.cprev, dE, e)) * 0.5;        // :41-43
                    const double R3 = fma(-sc.cprev, dE, fma(sc.invO, yl, On));  // :46
                    // sign(R3).*max(abs(R3)-thr,0) as R3 - clamp(R3,-thr,thr)
                    // (thr >= 0): |R3| > thr gives R3 -/+ thr, the same rounded
                    // difference; otherwise a zero; NaN and Inf pass through
                    const double Ev = R3 - fmin(fmax(R3, -sc.thr), sc.thr); // :47
                    const double rL = dL - On;                              // :50
                    const double rO = On - Ev;                              // :51
                    const double YLn = fma(sc.muL, rL, yl);                 // :52
                    const double Tn = fma(sc.invL_next, YLn, d - On);       // :33 (k+1)
                    // (Y_O^(k+1) = YLn - muO (E^(k+1) - E^(k)) is rebuilt by
                    // the next K5; :53 is never evaluated here)
                    // norm sums (:59): this kernel's own order (per lane, then
                    // a fixed tree), so fusing them costs no parity
                    ssL = fma(rL, rL, ssL);
                    ssO = fma(rO, rO, ssO);
                    En[r] = Ev;
                    YLn2[q] = YLn;
                    tr[r] = Tn;
                }
                bst(YLn2, rYL, tt, p);
                keep[p] = YLn2;
            }
            if constexpr (DE) {  // E^(k+1) over E^(k-1), densely
                __builtin_nontemporal_store(d2v{En[0], En[1]}, Ep2 + o);
                __builtin_nontemporal_store(d2v{En[2], En[3]}, Ep2 + o + 64);
                ++ndense;
            } else {
                ce_encode(En, lane, cs, rCEp, (int)(tt * 1024), Ep2, o, ndense);
            }
            keep[2] = d2v{En[0], En[1]};
            keep[3] = d2v{En[2], En[3]};
        }
        // T -> "TX" order (common.h): lane l, slot s holds T(ij = 4s+(l>>4), t = l&15)
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[(tg + 4 * r) * 17 + il] = tr[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            d2v tv;
            tv[0] = ts[il * 17 + 4 * (2 * p) + tg];
            tv[1] = ts[il * 17 + 4 * (2 * p + 1) + tg];
            bst(tv, rT, tt, p);
            keep[4 + p] = tv;
        }
        // Y_L and E data live until here (past the T transpose and stores)
        if (TRITD_STORE_KEEP) asm volatile("" ::"v"(keep[0]), "v"(keep[1]), "v"(keep[2]), "v"(keep[3]));
        // W^T(k, ij) += sum_t C^(t,k) T(t, ij): K-step r covers t = t0+4r+(l>>4);
        // the C/D register of T is directly the B operand
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m)
                wacc[m] = mfma4(opW(buf, r, m), tr[r], wacc[m]);
        // T data live until here (past the W MFMAs)
        if (TRITD_STORE_KEEP) asm volatile("" ::"v"(keep[4]), "v"(keep[5]));
        // the slice SD t-tiles ahead into the buffer read SD t-tiles ago
        if (ps) stage_store(slice_buf(tt + SD - t0));
        if (bar) __syncthreads();
        // step boundary: the scheduler would otherwise hoist the next step's
        // work above the barrier
        __builtin_amdgcn_sched_barrier(0);
    };

    Regs xa, xb;
#pragma unroll
    for (int q = 0; q < (PRO ? 3 : 2); ++q)
        xa.x[q][0] = xa.x[q][1] = xb.x[q][0] = xb.x[q][1] = d2v{0.0, 0.0};
    xa.ed[0] = xa.ed[1] = xb.ed[0] = xb.ed[1] = d2v{0.0, 0.0};
    xa.edp[0] = xa.edp[1] = xb.edp[0] = xb.edp[1] = d2v{0.0, 0.0};
    xa.ce = xb.ce = xa.cep = xb.cep = 0.0;
    // Prologue, in issue order: the first SD C^ slices (L2), the first tile
    // and slots (HBM), then the Khatri-Rao gather (L2).  vmcnt is in order,
    // so the slices' LDS writes wait for the slices only, and no L2 round
    // trip is waited for before the HBM loads are in flight.  Every KR load
    // is unconditional (an inactive wave's i = j = 0 is in range; its KR is
    // zeroed by a select): loads guarded by `active` compiled to a branch and
    // a vmcnt(0) wait per element, KS serial L2 round trips at the start of
    // every workgroup (round 6).
    static_assert(SD >= 1 && SD <= 2, "k5_fused: the prologue stages at most two slices");
    d2v sv1[NS];
    const bool st0 = t0 < t1, st1 = SD > 1 && t0 + 1 < t1;
    if (st0) stage_load_to(t0, sv);
    if (st1) stage_load_to(t0 + 1, sv1);
    load_slot(t0, xa);
    load_slot(t0 + 1, xb);
    if (PF) {
        load(t0, xa);
        if (DE) {
            load_dense(t0, xa);
            load_dense_p(t0, xa);
        }
    }
    double av[KS], bv[KS];
    if (!PRO) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + tg;
            av[s] = a.Ah[j * a.ahj + i * RP + k];
            bv[s] = a.Bh[j * a.bhj + k];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (st0) stage_store_from(slice_buf(0), sv);
    if (st1) stage_store_from(slice_buf(1), sv1);
    __syncthreads();
    if (!PRO) {
#pragma unroll
        for (int s = 0; s < KS; ++s) kr[s] = active ? av[s] * bv[s] : 0.0;
    }
    int64_t tt = t0;
    // steps in pairs (the register sets alternate by name; every flag is a
    // constant inside the loop); with SD = 2 only the second step of a pair
    // ends at a barrier
    // (SD = 1, A/B only: every step ends at a barrier)
    for (; tt + 3 < t1; tt += 2) {
        body(tt, slice_buf(tt - t0), xa, xb, true, true, SD == 1);
        body(tt + 1, slice_buf(tt + 1 - t0), xb, xa, true, true, true);
    }
    {
        const int64_t rem = t1 - tt;  // 1..3 steps left
        body(tt, slice_buf(tt - t0), xa, xb, rem > 1, rem > SD, SD == 1 && rem > 1);
        if (rem > 1) body(tt + 1, slice_buf(tt + 1 - t0), xb, xa, rem > 2, rem > 1 + SD, rem > 2);
        if (rem > 2) body(tt + 2, slice_buf(tt + 2 - t0), xa, xb, false, false, false);
    }
    // Epilogue lane values recomputed here from threadIdx (opaque to the
    // compiler): otherwise it hoists the W addresses and lane tests above the
    // walk and keeps them live through it, spilling 11 VGPRs (stored and
    // reloaded once per wave: 46 MB each way per launch at 512^3, round 3 PMC)
    int lane_e = (int)threadIdx.x;
    asm volatile("" : "+v"(lane_e));
    lane_e &= 63;
    if (tile < a.tiles) {
        // W^T C/D layout: row k = 16m + tg + 4rr, col ij = il; a t-split walk
        // writes its chunk's partial W into set `chunk` (summed by k_w_reduce)
        const int il_e = lane_e & 15, tg_e = lane_e >> 4;
        double* wp = a.Wk + (tile << 4) + il_e + chunk * (int64_t)RP * a.plane + (int64_t)tg_e * a.plane;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                wp[(int64_t)(16 * m + 4 * rr) * a.plane] = wacc[m][rr];
    }

    if (!PRO && ndense && lane_e == 0)  // spread over DENSE_SLOTS counters
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
        if (lane_e == 0) {
            red[0][wid] = ssL;
            red[1][wid] = ssO;
        }
        __syncthreads();
        if (lane_e == 0 && wid == 0) {
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
// almost idle, so the walk is cut into chunks of >= 4 t-tiles until there are
// about 256 workgroups; each chunk's W is a partial set that M1 / M2 sum as
// they read W.  (Config 2, round 4: 18 chunks of 4 against 9 of 8, iteration
// 0.106 vs 0.114 ms; 36 of 2: 0.113 ms — tools/rounds/r4/round4_c2_tsplit.sh.)
int k5_tsplit(const Geom& g) {
    if (g.RP > 64) return 1;
    const int64_t wg = cdiv(g.tiles, K5_WAVES);
    const int64_t smax = g.ntt / 4 > 1 ? g.ntt / 4 : 1;  // chunks of >= 4 t-tiles
    if (const char* e = std::getenv("TRITD_K5_TSPLIT")) {  // override (read once per session)
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


void launch_k5(const Geom& g, const K5Args& a, bool prologue, hipStream_t st, bool dense_e) {
    if (a.side.on && (prologue || g.RP > 64)) throw Error(TRITD_ERR_ARG, "K5 side solve: RP <= 64 only");
    if (dense_e && (prologue || g.RP > 64)) throw Error(TRITD_ERR_ARG, "K5 dense-E mode: RP <= 64");
    K5Args b = a;  // (the macro below launches with `b`)
    b.tsplit = g.tsplit;  // fixed at session creation (solver.cpp)
    const dim3 grid(k5_grid(g) * b.tsplit + (a.side.on ? 1 : 0)), block(64 * K5_WAVES);
#define K5_CASE(RPV)                                                                       \
    case RPV:                                                                              \
        if (prologue)                                                                      \
            hipLaunchKernelGGL((k5_fused<RPV, true>), grid, block, 0, st, b);              \
        else if (dense_e && RPV <= 64)                                                     \
            hipLaunchKernelGGL((k5_fused<RPV, false, (RPV <= 64)>), grid, block, 0, st, b); \
        else                                                                               \
            hipLaunchKernelGGL((k5_fused<RPV, false>), grid, block, 0, st, b);             \
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
    // a t-split walk leaves W as partial sets: the CP model's M1 / M2 sum them
    // as they read W (k_contract.hip); the Qi model's contractions read one W,
    // summed here in set order
    if (b.tsplit > 1 && a.ahj != 0) {
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

__global__ void k_finish(const double* ss, double normD, int k, double tol, double* errHist,
                         double* errL, double* errO, int* ctrl, int single) {
    if (ctrl[0]) return;
    finish_body(ss, normD, k, tol, errHist, errL, errO, ctrl, single);
}

// clear: zero the pairs after reading them (each thread clears the pairs it
// read).  The sharded schedule's norm partials live in red1_'s tail, sized to
// the largest shard's K5 grid; a rank with fewer workgroups leaves the slots
// past its own at zero, and the all-reduce writes sums into all of them.
__global__ __launch_bounds__(256) void k_reduce_finish(FinishArgs f) { reduce_finish_wg<256>(f); }

void launch_reduce_finish(double* partial, int n, double normD, int k, double tol,
                          double* errHist, double* errL, double* errO, int* ctrl, bool single,
                          hipStream_t st, bool clear) {
    FinishArgs f;
    f.p = partial; f.n = n; f.normD = normD; f.k = k; f.tol = tol;
    f.errHist = errHist; f.errL = errL; f.errO = errO; f.ctrl = ctrl;
    f.single = (int)single; f.clear = (int)clear; f.on = 1;
    hipLaunchKernelGGL(k_reduce_finish, dim3(1), dim3(256), 0, st, f);
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

// Placement probe: K5's HBM pattern (read D, Y_L and the tile's 256 B
// compact-E slot; write Y_L in place, T and the slot; one wave per ij-tile
// walking its t-tiles, prefetched) without the arithmetic.  K5 is HBM-bound
// and its bandwidth depends on where the pool landed physically; the session
// times candidate pools with this and keeps the fastest.
// Contents are overwritten with garbage.
__global__ __launch_bounds__(256) void k_pool_probe(double* D, double* YL, double* T, double* CE,
                                                    int64_t tiles4, int64_t ntt) {
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= tiles4) return;
    d2v* P[3] = {reinterpret_cast<d2v*>(D), reinterpret_cast<d2v*>(YL), reinterpret_cast<d2v*>(T)};
    auto tb = [&](int64_t tt) { return tm_tile_base(tile, tt, ntt); };
    struct R {
        d2v x[2][2];
        double ce;
    };
    R xa, xb;
    auto load = [&](int64_t tt, R& nx) {
        const int64_t o = (tb(tt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int f = 0; f < 2; ++f) nx.x[f][p] = P[f][o + 64 * p];
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
            P[1][o + 64 * p] = c.x[0][p] + c.x[1][p];
            P[2][o + 64 * p] = c.x[0][p] - c.x[1][p];
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

void launch_pool_probe(const Geom& g, double* D, double* YL, double* T, double* CE, hipStream_t st) {
    hipLaunchKernelGGL(k_pool_probe, dim3((unsigned)(g.tiles4 / 4)), dim3(256), 0, st, D, YL, T, CE,
                       g.tiles4, g.ntt);
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
