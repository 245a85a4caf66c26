// K5 for data of class single (fp32 path) and its companions.
//
// Same fused update as k_admm.hip (triple_decomp_ADMM.m:38-53, next :33,
// W = T x3 C^), evaluated under MATLAB's class rules for a single D: every
// elementwise statement in single with the double scalars rounded to single
// (IterScalars32), L from v_mfma_f32_16x16x4_f32 (MATLAB: double L rounded to
// single where it meets D), W in single.  RP in {16, 32, 48, 64, 128, 256}.
//
// fp32 tile layout (one 16 x 16 TM tile = 256 floats = 1 KB): lane l holds
// the four consecutive t = 4*(l>>4) + r (r = 0..3) of row i = l & 15 at
// floats 4l..4l+3 -- the C/D map of the f32 16x16 MFMA (row = 4*(lane>>4) +
// reg, col = lane & 15), so a tile moves with ONE dwordx4 per lane.  T is
// stored in the TX order of the mode-3 MFMA operand: lane l, slot s holds
// T(ij = 4s + (l>>4), t = l & 15) at float 4l + s.
//
// Compact E (fp32): one 64-float (256 B) slot per tile, lane l holding word
// l: words 0..49 the nonzeros in (w, lane) order, bytes 200..249 their tile
// positions 4 lane + w, word 63 the count; more than 50 nonzeros -> the tile
// is stored densely in E and its count is all ones (ce32_decode below).
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "kernels.h"

namespace tritd {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
static constexpr int K5W = 4;
// Compact-E slot (fp32): words 0..49 the nonzero values in (w, l) order,
// bytes CE32_IDX_BYTE + q (words 50..62) their tile positions 4 l + w (the f4
// order a lane holds), word 63 the count (all ones: dense).  Decoding
// scatters the values into a per-wave LDS tile image (k_admm.hip: ce_decode).
constexpr int CE32_CAP = 50;
constexpr int CE32_IDX_BYTE = 4 * CE32_CAP;  // 200
constexpr int CE32_CNT_WORD = 63;
constexpr int CE32_IMG = 256 + 64;

bool rp_supported32(int RP) {
    return RP == 16 || RP == 32 || RP == 48 || RP == 64 || RP == 128 || RP == 256;
}
int padded_rank32(int R) {
    if (R <= 64) return (int)round_up(R, 16);
    return R <= 128 ? 128 : 256;
}

__device__ __forceinline__ f4 mfma32(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float sign32(float x) {  // MATLAB sign, select-only
    const float s = x == 0.0f ? 0.0f : __builtin_copysignf(1.0f, x);
    return __builtin_isnan(x) ? x : s;
}
__device__ __forceinline__ int lanes_below32(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ bool ce32_is_dense(float sv) {
    return (uint32_t)__builtin_amdgcn_readlane(__float_as_int(sv), CE32_CNT_WORD) == 0xFFFFFFFFu;
}
__device__ __forceinline__ bool lane_bit32(uint64_t m, int lane) {
    (void)lane;
    return __builtin_amdgcn_inverse_ballot_w64(m);  // the uniform mask as the lane condition
}
// this lane's 4 elements from its slot word sv through the wave's LDS tile
// image img (CE32_IMG floats, zero on entry and on return): lane q < count
// writes value q at its position, every lane reads its f4, the writers zero
// their position again; true for a dense tile
__device__ __forceinline__ bool ce32_decode(float sv, int lane, float* img, float (&e)[4]) {
    const int b = __float_as_int(sv);
    const uint32_t cnt = (uint32_t)__builtin_amdgcn_readlane(b, CE32_CNT_WORD);
    const int src = (CE32_IDX_BYTE / 4 + (lane >> 2)) << 2;  // word holding byte `lane` (lane-constant)
    const uint32_t wd = (uint32_t)__builtin_amdgcn_ds_bpermute(src, b);
    const int pos = (int)__builtin_amdgcn_ubfe(wd, 8 * (lane & 3), 8);
    const int at = ((uint32_t)lane < cnt && cnt <= (uint32_t)CE32_CAP) ? pos : 256 + lane;
    img[at] = sv;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const f4 v = *reinterpret_cast<const f4*>(img + 4 * lane);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    img[at] = 0.0f;
#pragma unroll
    for (int w = 0; w < 4; ++w) e[w] = v[w];
    return cnt == 0xFFFFFFFFu;
}
// store this lane's 4 elements as the tile's slot (every lane one word), or
// densely (wave-uniform, rare) when they do not fit.  cs: 128-float per-wave
// LDS image (slot + junk area for the zeros: no divergent branch)
__device__ __forceinline__ void ce32_encode(const float (&En)[4], int lane, float* cs,
                                            float* slot, f4* Etile,
                                            unsigned& ndense) {
    uint64_t nz[4];
    int cnt = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        nz[w] = __ballot(En[w] != 0.0f);
        cnt += __builtin_popcountll(nz[w]);
    }
    const bool dense = cnt > CE32_CAP;
    cs[lane] = 0.0f;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    unsigned char* cb = reinterpret_cast<unsigned char*>(cs);
    int pre = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const bool bit = !dense && lane_bit32(nz[w], lane);
        const int at = pre + lanes_below32(nz[w]), away = 64 + lane;
        cs[bit ? at : away] = En[w];
        cb[bit ? CE32_IDX_BYTE + at : 4 * away + w] = (unsigned char)(4 * lane + w);
        pre += __builtin_popcountll(nz[w]);
    }
    if (lane == 0) cs[CE32_CNT_WORD] = __int_as_float(dense ? -1 : cnt);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const float v = cs[lane];
    if (dense) {
        Etile[lane] = f4{En[0], En[1], En[2], En[3]};
        ++ndense;  // wave-uniform; one atomic per wave at the end (a per-tile
                   // atomic on one counter serialised: 17 -> 53 ms once E turned dense)
    }
    slot[lane] = v;
}

// Register budget: two waves per SIMD up to RP = 128; at RP = 256 the L
// operands (64) + W accumulators (64) + two tile sets (34) + C^ staging (16)
// + L accumulators do not fit 256, and the kernel runs one wave per SIMD
// (config 5 is MFMA-bound: 128 MFMAs per tile).
template <int RP, bool PRO>
__global__ __launch_bounds__(64 * K5W) __attribute__((amdgpu_waves_per_eu(RP >= 256 ? 1 : 2, 2)))
void k5_f32(K5Args32 a) {
    if (*a.stop) return;
    constexpr int KS = RP / 4;    // MFMA K-steps of L
    constexpr int MT = RP / 16;   // k-tiles of W
    constexpr int LDC = RP + 4;   // [t][k] row stride: the 4 t-groups of a read fall in distinct banks
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int il = lane & 15;
    const int tg = lane >> 4;
    const int64_t tile = (int64_t)blockIdx.x * K5W + wid;
    const bool active = tile < a.tiles;
    const int64_t qper = a.n1p >> 4;
    const int64_t j = active ? tile / qper : 0;
    const int64_t i = active ? ((tile - j * qper) << 4) + il : 0;
    const int64_t ntt = a.ntt;

    // C^ slice of the t-tile, [t][k] rows of stride LDC.  The L operand's K
    // index is renumbered k = (l>>4) * KS + s, so lane l walks its row
    // t0 + (l&15) contiguously and reads four K-steps per ds_read_b128 (row
    // offsets il * LDC put the 16 lanes of a group on distinct banks).
    // WB (RP % 64 == 0): W's M index is renumbered too, M-tile m row rho <->
    // k = rho * MT + m, so lane l reads the MT contiguous k of chunk (l&15) of
    // row t0 + 4(l>>4) + r with MT/4 ds_read_b128; inside each chunk of
    // G = MT/4 16-byte granules, granule q sits at (q + (c*G >> 4)) mod G,
    // which puts the 16 chunks a W read touches on 16 distinct bank groups
    // and keeps the L reads conflict-free.  Otherwise W reads C^(t, 16m + l&15)
    // one float per MFMA.
    constexpr bool WB = RP % 64 == 0;
    constexpr int G = WB ? MT / 4 : 1;
    auto gran = [](int c, int q) { return c * G + ((q + ((c * G) >> 4)) & (G - 1)); };
    __shared__ __attribute__((aligned(16))) float sC[2][16 * LDC];
    __shared__ float tsm[K5W][16 * 17]; // per-wave T transpose
    __shared__ float csm[K5W][128];     // per-wave compact-E slot image
    __shared__ __attribute__((aligned(16))) float cimg[PRO ? 1 : K5W][CE32_IMG];  // decode images
    float* ts = tsm[wid];
    float* cs = csm[wid];
    if (!PRO) {
        for (int q = lane; q < CE32_IMG; q += 64) cimg[wid][q] = 0.0f;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
    // every __shared__ array of this kernel (sC, tsm, csm, the W exchange wl,
    // red), in bytes: at most the 160 KiB of a CU
    static_assert(sizeof(float) * (2 * 16 * LDC + K5W * 16 * 17 + K5W * 128 + K5W * (RP * 16 + 16) +
                                   (PRO ? 1 : K5W) * CE32_IMG) +
                          sizeof(double) * 2 * K5W <=
                      160 * 1024,
                  "k5_f32: LDS over the 160 KiB of a CU");

    // C^ slice of one t-tile: 16 rows x RP floats, loaded before the tile
    // prefetch, written to LDS after the tile's compute (in-order vmcnt)
    constexpr int SQ = 16 * RP / 4;
    constexpr int NS = (SQ + 64 * K5W - 1) / (64 * K5W);
    f4 sv[NS];
    auto stage_load = [&](int64_t tt) {
        const f4* src = reinterpret_cast<const f4*>(a.ChF + (tt << 4) * RP);
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5W;
            if (SQ % (64 * K5W) == 0 || e < SQ) sv[q] = src[e];
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5W;
            if (SQ % (64 * K5W) == 0 || e < SQ) {
                const int row = (4 * e) / RP, k = (4 * e) % RP;
                const int kp = WB ? 4 * gran((k >> 2) / G, (k >> 2) % G) : k;
                *reinterpret_cast<f4*>(&sC[buf][row * LDC + kp]) = sv[q];
            }
        }
    };

    float kr[KS];  // L operand KR(ij = l & 15, k = (l>>4) * KS + s), single-rounded
    if (!PRO) {
        // unconditional loads, all issued first (k_admm.hip: the KR gather)
        double av[KS], bv[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = tg * KS + s;
            av[s] = a.Ah[i * RP + k];
            bv[s] = a.Bh[j * RP + k];
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) kr[s] = active ? (float)(av[s] * bv[s]) : 0.0f;
    }
    f4 wacc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) wacc[m] = f4{0.0f, 0.0f, 0.0f, 0.0f};

    double ssL = 0.0, ssO = 0.0;
    unsigned ndense = 0;  // E tiles of this wave stored densely (wave-uniform)
    const IterScalars32 sc = a.s;
    const f4* D4 = reinterpret_cast<const f4*>(a.D);
    f4* O4 = reinterpret_cast<f4*>(a.O);
    f4* E4 = reinterpret_cast<f4*>(a.E);
    f4* YL4 = reinterpret_cast<f4*>(a.YL);
    f4* YO4 = reinterpret_cast<f4*>(a.YO);
    f4* T4 = reinterpret_cast<f4*>(a.T);

    // two register sets, unrolled by two (no cur = next copies); slots two
    // tiles ahead so a dense tile is known when its batch is issued; the only
    // branches are wave-uniform and rare (see k_admm.hip)
    struct Regs {
        f4 x[3];  // D, Y_L, Y_O (PRO: O)
        f4 ed;    // dense E (overflowed tile only)
        float ce; // this lane's slot word
    };
    auto tbase = [&](int64_t tt) { return tm_tile_base(tile, tt, ntt); };
    auto load = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tbase(tt) >> 2) + lane;
        nx.x[0] = D4[o];
        nx.x[1] = YL4[o];
        nx.x[2] = (PRO ? O4 : YO4)[o];
    };
    auto load_dense = [&](int64_t tt, Regs& nx) { nx.ed = E4[(tbase(tt) >> 2) + lane]; };
    auto load_slot = [&](int64_t tt, float& ce) {
        const int64_t t2 = tt < ntt ? tt : ntt - 1;
        ce = a.CE[(tbase(t2) >> 8) * CE32_SLOT + lane];
    };
    auto body = [&](int64_t tt, int buf, Regs& cx, Regs& nx, bool pf) {
        const int64_t tb = tbase(tt);
        const int64_t o = (tb >> 2) + lane;
        if (pf) {
            const bool dn1 = PRO ? false : ce32_is_dense(nx.ce);
            stage_load(tt + 1);
            load(tt + 1, nx);
            __builtin_amdgcn_sched_barrier(0);
            if (!PRO && dn1) load_dense(tt + 1, nx);
        }
        float ev[4];
        if (!PRO) {
            const bool dn = ce32_decode(cx.ce, lane, cimg[PRO ? 0 : wid], ev);
#pragma unroll
            for (int r = 0; r < 4; ++r) ev[r] = dn ? cx.ed[r] : ev[r];
            if (pf) load_slot(tt + 2, cx.ce);
        }
        const float* cR = sC[buf];
        float tr[4];
        if (PRO) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float d = cx.x[0][r], yl = cx.x[1][r], ov = cx.x[2][r];
                tr[r] = (d - ov) + sc.invL * yl;  // :33
            }
        } else {
            f4 lacc[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) lacc[q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
            const f4* cL = reinterpret_cast<const f4*>(cR + il * LDC);
#pragma unroll
            for (int s4 = 0; s4 < KS / 4; ++s4) {
                // logical granule tg * KS/4 + s4 of row il
                const int gl = tg * (KS / 4) + s4;
                const f4 c = cL[WB ? gran(gl / G, gl % G) : gl];
#pragma unroll
                for (int u = 0; u < 4; ++u) lacc[u] = mfma32(c[u], kr[4 * s4 + u], lacc[u]);
            }
            const f4 Lv = (lacc[0] + lacc[1]) + (lacc[2] + lacc[3]);
            float En[4];
            f4 YLn, YOn;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float d = cx.x[0][r], yl = cx.x[1][r], yo = cx.x[2][r], e = ev[r];
                const float L = Lv[r];
                const float R1 = (d - L) + sc.invL * yl;               // :41
                const float R2 = e - sc.invO * yo;                     // :42
                // x/den as reciprocal product + exact-residual FMA correction,
                // sign()*max() as R3 - clamp(R3,-thr,thr): fewer VALU ops (k_admm.hip)
                const float Onum = sc.muL * R1 + sc.muO * R2;
                const float q0 = Onum * sc.rden;
                const float On = fmaf(fmaf(-q0, sc.den, Onum), sc.rden, q0);  // :43
                const float R3 = On + sc.invO * yo;                    // :46
                const float Ev = R3 - fminf(fmaxf(R3, -sc.thr), sc.thr);  // :47
                const float rL = (d - L) - On;                         // :50
                const float rO = On - Ev;                              // :51
                const float yln = yl + sc.muL * rL;                    // :52
                const float yon = yo + sc.muO * rO;                    // :53
                tr[r] = (d - On) + sc.invL_next * yln;                 // :33 (k+1)
                ssL = fma((double)rL, (double)rL, ssL);
                ssO = fma((double)rO, (double)rO, ssO);
                En[r] = Ev;
                YLn[r] = yln;
                YOn[r] = yon;
            }
            YL4[o] = YLn;
            YO4[o] = YOn;
            ce32_encode(En, lane, cs, a.CE + (tb >> 8) * CE32_SLOT, E4 + (tb >> 2), ndense);
        }
        // T -> TX order through the wave's LDS tile: ts[t][ij]
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[(4 * tg + r) * 17 + il] = tr[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        f4 tv;
#pragma unroll
        for (int s = 0; s < 4; ++s) tv[s] = ts[il * 17 + 4 * s + tg];
        T4[o] = tv;
        // W^T(k, ij) += sum_t C^(t,k) T(t,ij): K-step r covers t = 4(l>>4) + r
        if (WB) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f4* cW = reinterpret_cast<const f4*>(cR + (4 * tg + r) * LDC);
#pragma unroll
                for (int q = 0; q < G; ++q) {
                    const f4 c = cW[gran(il, q)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) wacc[4 * q + u] = mfma32(c[u], tr[r], wacc[4 * q + u]);
                }
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    wacc[m] = mfma32(cR[(4 * tg + r) * LDC + 16 * m + il], tr[r], wacc[m]);
        }
        if (pf) stage_store(buf ^ 1);
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
    };

    Regs xa, xb;
#pragma unroll
    for (int q = 0; q < 3; ++q) xa.x[q] = xb.x[q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    xa.ed = xb.ed = f4{0.0f, 0.0f, 0.0f, 0.0f};
    xa.ce = xb.ce = 0.0f;
    if (!PRO) {
        load_slot(0, xa.ce);
        load_slot(1, xb.ce);
    }
    load(0, xa);
    if (!PRO && ce32_is_dense(xa.ce)) load_dense(0, xa);
    stage_load(0);
    stage_store(0);
    __syncthreads();
    int64_t tt = 0;
    for (; tt + 2 < ntt; tt += 2) {
        body(tt, 0, xa, xb, true);
        body(tt + 1, 1, xb, xa, true);
    }
    if (tt + 1 < ntt) {
        body(tt, 0, xa, xb, true);
        body(tt + 1, 1, xb, xa, false);
    } else {
        body(tt, 0, xa, xb, false);
    }
    {
        // W out through LDS: a wave's 16 ij of a k-plane are 64 B, half an
        // L2 line, and partial-line stores from four waves cost a line read +
        // write each (K5 traffic 1.32x algorithmic at config 5).  The four
        // waves hold four adjacent ij-tiles = 64 consecutive ij, so after the
        // exchange every store is one 256 B row of a plane.  W^T C/D layout
        // (f32): M-tile m row rho = 4(l>>4) + rr, col ij = l & 15;
        // k = rho * MT + m (WB) or 16m + rho.
        constexpr int WS = RP * 16 + 16;  // per-wave stride (pad: the read rows hit distinct banks)
        __shared__ float wl[K5W * WS];
        __syncthreads();  // sC / tsm reads of the last tile are done
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int rho = 4 * tg + rr;
                const int k = WB ? rho * MT + m : 16 * m + rho;
                wl[wid * WS + k * 16 + il] = wacc[m][rr];
            }
        __syncthreads();
        const int64_t t0 = (int64_t)blockIdx.x * K5W;      // first tile of the block
        const int lw = lane >> 4;                           // source wave of this lane
        const bool ok = t0 + lw < a.tiles;
        float* dst = a.Wk + (t0 << 4) + lane;
#pragma unroll 4
        for (int k = wid; k < RP; k += K5W)
            if (ok) dst[(int64_t)k * a.plane] = wl[lw * WS + k * 16 + il];
    }
    if (!PRO && ndense && lane == 0)  // spread over DENSE_SLOTS counters
        atomicAdd(a.dense_tiles + ((blockIdx.x * K5W + wid) & (DENSE_SLOTS - 1)),
                  (unsigned long long)ndense);
    if (!PRO) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            ssL += __shfl_xor(ssL, off);
            ssO += __shfl_xor(ssO, off);
        }
        __shared__ double red[2][K5W];
        if (lane == 0) {
            red[0][wid] = ssL;
            red[1][wid] = ssO;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double x = 0.0, y = 0.0;
            for (int w = 0; w < K5W; ++w) {
                x += red[0][w];
                y += red[1][w];
            }
            a.partial[2 * blockIdx.x] = x;
            a.partial[2 * blockIdx.x + 1] = y;
        }
    }
}

// RP = 256 with the rank split over a wave pair (the default there): two
// waves share each ij-tile, wave h of the pair holding the K-steps
// s in [h*KS/2, (h+1)*KS/2) of the L operand (k = (l>>4) * KS + s) and the
// W M-tiles m = 4q + u of granules q in [0, GH0) (h = 0) or [GH0, G) (h = 1).
// Per t-tile each forms its half of L, the pair adds the halves through LDS
// (both in the same order: both waves then hold bitwise the same L), wave 0
// runs the elementwise chain (stores Y_L, Y_O, T, E and sums the norms), and
// each accumulates its W M-tiles.  Half the L operands and part of the W
// accumulators per wave fit two waves per SIMD, which the one-wave kernel (352 VGPRs) could
// not: at one wave per SIMD a t-tile step took ~8 800 cycles against ~5 200
// of issue.
template <int RP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k5_f32s(K5Args32 a) {
    static_assert(RP == 256, "k5_f32s: RP = 256 (the L-read permutation assumes 4 granules per group)");
    if (*a.stop) return;
    constexpr int KS = RP / 4, MT = RP / 16, LDC = RP + 4;
    constexpr int G = MT / 4, KSH = KS / 2;
    // W granules (of 4 M-tiles) of the h = 0 wave, which also runs the
    // elementwise chain; h = 1 holds the other G - GH0 (round 5: 1 of 4 vs
    // 2 of 4: K5 13.65 vs 13.75 ms; the L K-steps split 4:12 or 12:4 instead
    // of 8:8: 14.00 / 14.02 ms — profiles/round5/ab_k5_split.txt; with the
    // roles alternated per round below, 1 : 3 is 13.39 ms and 2 : 2 13.82)
    constexpr int GH0 = 1;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int slot = wid >> 1;  // ij-tile of the pair within the workgroup
    const int il = lane & 15, tg = lane >> 4;
    const int64_t tile = (int64_t)blockIdx.x * 2 + slot;
    const bool active = tile < a.tiles;
    const int64_t qper = a.n1p >> 4;
    const int64_t j = active ? tile / qper : 0;
    const int64_t i = active ? ((tile - j * qper) << 4) + il : 0;
    const int64_t ntt = a.ntt;
    auto gran = [](int c, int q) { return c * G + ((q + ((c * G) >> 4)) & (G - 1)); };
    // Deferred W: the h = 1 wave runs the W MFMAs of tile tt-1 during step tt
    // (beside the chain of tt on its partner), from a T transpose buffer and a
    // C^ slice one step old: no barrier between the chain and W, three C^
    // slices (tt-1 in use by h = 1, tt, tt+1 being staged) and two transpose
    // buffers (round 3: K5 15.49 -> 15.24 ms, iteration 22.23 -> 21.95 ms)
    constexpr int NSL = 3;
    __shared__ __attribute__((aligned(16))) float sC[NSL][16 * LDC];
    __shared__ float tsm[2][2][16 * 17];
    __shared__ float csm[2][128];
    __shared__ __attribute__((aligned(16))) float cimg[4][CE32_IMG];  // per-wave decode images
    __shared__ __attribute__((aligned(16))) f4 lx[2][2][64];  // [slot][half] partial L
    float* cs = csm[slot];
    for (int q = lane; q < CE32_IMG; q += 64) cimg[wid][q] = 0.0f;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    constexpr int WS = RP * 16 + 16;
    static_assert(2 * WS <= 2 * 16 * LDC, "k5_f32s: the W exchange reuses the C^ slices");

    constexpr int SQ = 16 * RP / 4;
    constexpr int NS = SQ / 256;
    static_assert(SQ % 256 == 0, "k5_f32s: staging");
    f4 sv[NS];
    auto stage_load = [&](int64_t tt) {
        const f4* src = reinterpret_cast<const f4*>(a.ChF + (tt << 4) * RP);
#pragma unroll
        for (int q = 0; q < NS; ++q) sv[q] = src[threadIdx.x + q * 256];
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 256;
            const int row = (4 * e) / RP, k = (4 * e) % RP;
            *reinterpret_cast<f4*>(&sC[buf][row * LDC + 4 * gran((k >> 2) / G, (k >> 2) % G)]) = sv[q];
        }
    };
    const IterScalars32 sc = a.s;
    const f4* D4 = reinterpret_cast<const f4*>(a.D);
    f4* E4 = reinterpret_cast<f4*>(a.E);
    f4* YL4 = reinterpret_cast<f4*>(a.YL);
    f4* YO4 = reinterpret_cast<f4*>(a.YO);
    f4* T4 = reinterpret_cast<f4*>(a.T);
    struct Regs {
        f4 x[3];
        f4 ed;
        float ce;
    };
    auto tbase = [&](int64_t tt) { return tm_tile_base(tile, tt, ntt); };
    auto load = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tbase(tt) >> 2) + lane;
        nx.x[0] = D4[o];
        nx.x[1] = YL4[o];
        nx.x[2] = YO4[o];
    };
    auto load_dense = [&](int64_t tt, Regs& nx) { nx.ed = E4[(tbase(tt) >> 2) + lane]; };
    auto load_slot = [&](int64_t tt, float& ce) {
        const int64_t t2 = tt < ntt ? tt : ntt - 1;
        ce = a.CE[(tbase(t2) >> 8) * CE32_SLOT + lane];
    };
    double ssL = 0.0, ssO = 0.0;
    unsigned ndense = 0;
    // (Splitting the pair by role instead — one wave all of L and the chain,
    // the other all of W — measured 16.03 vs 15.22 ms, round 3.)

    // the walk, specialised per half (straight-line code in each)
    auto walk = [&](auto HC) {
        constexpr int h = decltype(HC)::value;
        constexpr int NKR = KSH;  // KR operands this wave holds
        constexpr int NG = h ? G - GH0 : GH0;  // W granules of this wave
        constexpr int NWT = 4 * NG;            // W M-tiles this wave accumulates
        f4 wacc[NWT];
        // KR(ij = l & 15, k), single-rounded, for the k this lane's L read
        // takes at slot s = 4 s4 + u: granule s4 of its half, permuted within
        // each group of 4 granules by the lane's K group tg (sig below), so
        // that the 16 lanes of a ds_read_b128 group hit 16 distinct 16-B bank
        // slots (the unpermuted order was 2-way conflicted: the gran rotation
        // below depends on tg).  Every k is still taken once; only which k
        // share an MFMA changes (the f32 sum of L is formed in another order).
        auto sig = [&](int s4) { return 4 * (s4 >> 2) + (((s4 & 3) - tg) & 3); };
        float kr[NKR];
        // gathered after the walk's first loads are issued (below): the
        // four consecutive k of each granule as two 16-byte loads per factor
        auto gather_kr = [&] {
            const d2v* ah = reinterpret_cast<const d2v*>(a.Ah + (active ? i : 0) * RP);
            const d2v* bh = reinterpret_cast<const d2v*>(a.Bh + (active ? j : 0) * RP);
#pragma unroll
            for (int s4 = 0; s4 < NKR / 4; ++s4) {
                const int k0 = (tg * KS + h * KSH + 4 * sig(s4)) >> 1;  // d2v index
                const d2v a0 = ah[k0], a1 = ah[k0 + 1], b0 = bh[k0], b1 = bh[k0 + 1];
                kr[4 * s4 + 0] = active ? (float)(a0[0] * b0[0]) : 0.0f;
                kr[4 * s4 + 1] = active ? (float)(a0[1] * b0[1]) : 0.0f;
                kr[4 * s4 + 2] = active ? (float)(a1[0] * b1[0]) : 0.0f;
                kr[4 * s4 + 3] = active ? (float)(a1[1] * b1[1]) : 0.0f;
            }
        };
#pragma unroll
        for (int m = 0; m < NWT; ++m) wacc[m] = f4{0.0f, 0.0f, 0.0f, 0.0f};
        // only the h = 0 wave of the pair loads the tile, decodes E and runs
        // the elementwise chain (round 3: K5 15.73 -> 15.45 ms); the h = 1
        // wave takes T from the LDS transpose buffer a step later
        constexpr bool CHAIN = h == 0;
        // W^T += C^T T for this wave's M-tiles (granules q in [Q0, Q0 + NG))
        auto wmfma = [&](const float* cR, const float (&tr)[4]) {
            constexpr int NQ = NG, Q0 = h ? GH0 : 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f4* cW = reinterpret_cast<const f4*>(cR + (4 * tg + r) * LDC);
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const f4 c = cW[gran(il, Q0 + q)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) wacc[4 * q + u] = mfma32(c[u], tr[r], wacc[4 * q + u]);
                }
            }
        };
        auto body = [&](int64_t tt, int buf, int nbuf, Regs& cx, Regs& nx, bool pf) {
            float* ts = tsm[slot][(int)(tt & 1)];
            const int64_t tb = tbase(tt);
            const int64_t o = (tb >> 2) + lane;
            if (pf) {
                const bool dn1 = CHAIN ? ce32_is_dense(nx.ce) : false;
                stage_load(tt + 1);
                if (CHAIN) load(tt + 1, nx);
                __builtin_amdgcn_sched_barrier(0);
                if (CHAIN && dn1) load_dense(tt + 1, nx);
            }
            float ev[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            if (CHAIN) {
                const bool dn = ce32_decode(cx.ce, lane, cimg[wid], ev);
#pragma unroll
                for (int r = 0; r < 4; ++r) ev[r] = dn ? cx.ed[r] : ev[r];
                if (pf) load_slot(tt + 2, cx.ce);
            }
            const float* cR = sC[buf];
            const f4* cL = reinterpret_cast<const f4*>(cR + il * LDC);
            f4 Lv = f4{0.0f, 0.0f, 0.0f, 0.0f};
            {
                f4 lacc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) lacc[q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int s4 = 0; s4 < KSH / 4; ++s4) {
                    // granule gl = 16 tg + 8 h + sig(s4) lands at gran(gl/G, gl%G)
                    // = 16 tg + 8 h + s4: the permutation undoes the rotation
                    const f4 c = cL[tg * (KS / 4) + h * (KSH / 4) + s4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) lacc[u] = mfma32(c[u], kr[4 * s4 + u], lacc[u]);
                }
                lx[slot][h][lane] = (lacc[0] + lacc[1]) + (lacc[2] + lacc[3]);
                __syncthreads();
                Lv = lx[slot][0][lane] + lx[slot][1][lane];  // same order in both waves
            }
            float En[4], tr[4];
            f4 YLn, YOn;
#pragma unroll
            for (int r = 0; r < 4 && CHAIN; ++r) {
                const float d = cx.x[0][r], yl = cx.x[1][r], yo = cx.x[2][r], e = ev[r];
                const float L = Lv[r];
                const float R1 = (d - L) + sc.invL * yl;               // :41
                const float R2 = e - sc.invO * yo;                     // :42
                const float Onum = sc.muL * R1 + sc.muO * R2;
                const float q0 = Onum * sc.rden;
                const float On = fmaf(fmaf(-q0, sc.den, Onum), sc.rden, q0);  // :43
                const float R3 = On + sc.invO * yo;                    // :46
                const float Ev = R3 - fminf(fmaxf(R3, -sc.thr), sc.thr);  // :47
                const float rL = (d - L) - On;                         // :50
                const float rO = On - Ev;                              // :51
                const float yln = yl + sc.muL * rL;                    // :52
                const float yon = yo + sc.muO * rO;                    // :53
                tr[r] = (d - On) + sc.invL_next * yln;                 // :33 (k+1)
                if (h == 0) {
                    ssL = fma((double)rL, (double)rL, ssL);
                    ssO = fma((double)rO, (double)rO, ssO);
                }
                En[r] = Ev;
                YLn[r] = yln;
                YOn[r] = yon;
            }
            if (h == 0) {
                YL4[o] = YLn;
                YO4[o] = YOn;
                ce32_encode(En, lane, cs, a.CE + (tb >> 8) * CE32_SLOT, E4 + (tb >> 2), ndense);
#pragma unroll
                for (int r = 0; r < 4; ++r) ts[(4 * tg + r) * 17 + il] = tr[r];
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                f4 tv;
#pragma unroll
                for (int s = 0; s < 4; ++s) tv[s] = ts[il * 17 + 4 * s + tg];
                T4[o] = tv;
            }
            if constexpr (h == 1) {
                // W of tile tt-1: its T (written by the partner in step tt-1,
                // before that step's closing barrier) and its C^ slice
                if (tt > 0) {
                    const float* tp = tsm[slot][(int)((tt - 1) & 1)];
#pragma unroll
                    for (int r = 0; r < 4; ++r) tr[r] = tp[(4 * tg + r) * 17 + il];
                    wmfma(sC[(int)((tt + NSL - 1) % NSL)], tr);
                }
            } else {
                wmfma(cR, tr);
            }
            if (pf) stage_store(nbuf);
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
        };
        Regs xa, xb;
#pragma unroll
        for (int q = 0; q < 3; ++q) xa.x[q] = xb.x[q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
        xa.ed = xb.ed = f4{0.0f, 0.0f, 0.0f, 0.0f};
        // every first load in flight before the first wait: the slots, tile
        // 0, slice 0 and the Khatri-Rao gather (round 5: the gather used to
        // complete before tile 0's loads were issued)
        load_slot(0, xa.ce);
        load_slot(1, xb.ce);
        load(0, xa);
        stage_load(0);
        gather_kr();
        if (ce32_is_dense(xa.ce)) load_dense(0, xa);
        stage_store(0);
        __syncthreads();
        int64_t tt = 0;
        {
            // slices rotate over three buffers: tile tt in tt % 3
            int b0 = 0;
            for (; tt + 2 < ntt; tt += 2) {
                const int b1 = b0 == 2 ? 0 : b0 + 1, b2 = b1 == 2 ? 0 : b1 + 1;
                body(tt, b0, b1, xa, xb, true);
                body(tt + 1, b1, b2, xb, xa, true);
                b0 = b2;
            }
            const int b1 = b0 == 2 ? 0 : b0 + 1, b2 = b1 == 2 ? 0 : b1 + 1;
            if (tt + 1 < ntt) {
                body(tt, b0, b1, xa, xb, true);
                body(tt + 1, b1, b2, xb, xa, false);
            } else {
                body(tt, b0, b1, xa, xb, false);
            }
            if constexpr (h == 1) {  // the last tile's W (its T and slice are final: no staging after it)
                float tr[4];
                const float* tp = tsm[slot][(int)((ntt - 1) & 1)];
#pragma unroll
                for (int r = 0; r < 4; ++r) tr[r] = tp[(4 * tg + r) * 17 + il];
                wmfma(sC[(int)((ntt - 1) % NSL)], tr);
            }
        }
        // W^T C/D layout: M-tile m row rho = 4(l>>4) + rr, col ij = l & 15,
        // k = rho * MT + m; this wave's m = 4(Q0 + q) + u
        float* wl = &sC[0][0];  // the C^ slices are dead after the walk
        __syncthreads();
#pragma unroll
        for (int mq = 0; mq < NWT; ++mq)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int m = 4 * (h ? GH0 : 0) + mq;
                const int k = (4 * tg + rr) * MT + m;
                wl[slot * WS + k * 16 + il] = wacc[mq][rr];
            }
    };
    // (Walking pairs grid-stride in 512 persistent workgroups instead, to
    // save the turnover of 131 072 short-lived ones: K5 15.88 vs 13.79 ms,
    // profiles/round5/ab_c5_prologue_persistent.txt — dropped.)
    // Roles alternate between workgroups that share a CU, so that each SIMD
    // hosts one chain wave (h = 0) and one partner: blocks are dealt to the
    // XCDs by blockIdx mod 8, so the two resident on a CU have the same
    // blockIdx parity but sit one round of `slots` apart (and a retiring
    // workgroup is replaced by one a whole number of rounds later).  Round
    // 5: alternating by blockIdx parity put both chain waves of a CU on the
    // same two SIMDs (K5 13.57 vs 13.39 ms with the 1 : 3 W split; with 2 : 2
    // 13.68 vs 13.82 — profiles/round5/ab_k5_roles.txt)
    const int64_t rnd = a.slots > 0 ? (int64_t)blockIdx.x / a.slots : (int64_t)blockIdx.x;
    const int hrole = (wid & 1) ^ (int)(rnd & 1);
    if (hrole)
        walk(std::integral_constant<int, 1>{});
    else
        walk(std::integral_constant<int, 0>{});
    __syncthreads();
    {
        // two adjacent ij-tiles = 32 consecutive ij: one 128 B row piece of
        // each k-plane
        const int64_t t0 = (int64_t)blockIdx.x * 2;
        float* wl = &sC[0][0];
        // 16-B stores: 8 lanes per 128 B row piece, 8 k-rows per instruction
        // (a quarter of the store instructions of the 4-B form: round 6, K5
        // 13.45 -> 13.29 ms, profiles/round6/c5_w_store16_ab.txt)
        const int qq = lane & 7;
        const int sl = qq >> 2, c4 = (qq & 3) * 4;
        const bool ok = t0 + sl < a.tiles;
        float* dst = a.Wk + (t0 << 4) + 16 * sl + c4;
#pragma unroll 2
        for (int k0 = 8 * wid; k0 < RP; k0 += 32) {
            const int k = k0 + (lane >> 3);
            const f4 v = *reinterpret_cast<const f4*>(&wl[sl * WS + k * 16 + c4]);
            if (ok) *reinterpret_cast<f4*>(dst + (int64_t)k * a.plane) = v;
        }
    }
    if (hrole == 0 && ndense && lane == 0)
        atomicAdd(a.dense_tiles + ((blockIdx.x * 2 + slot) & (DENSE_SLOTS - 1)), (unsigned long long)ndense);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        ssL += __shfl_xor(ssL, off);
        ssO += __shfl_xor(ssO, off);
    }
    __shared__ double red[2][4];
    if (lane == 0) {
        red[0][wid] = ssL;  // exactly 0 for the h = 1 waves
        red[1][wid] = ssO;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // adding the h = 1 zeros is exact: the pair sum of the h = 0 waves
        a.partial[2 * blockIdx.x] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        a.partial[2 * blockIdx.x + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}

// RP = 256 runs the pair kernel (one-wave k5_f32<256>: 16.86 vs 16.30 ms, round 2)
bool k5_split32(const Geom& g) { return g.RP == 256; }
int k5_parts32(const Geom& g) { return k5_split32(g) ? (int)cdiv(g.tiles, 2) : k5_grid(g); }

void launch_k5_32(const Geom& g, const K5Args32& a, bool prologue, hipStream_t st) {
    if (!prologue && k5_split32(g)) {
        // CU count per device, cached (shard threads of a device set may race
        // to fill an entry: both store the same value)
        static std::atomic<int> cus[64];
        int dev = 0;
        TRITD_HIP(hipGetDevice(&dev));
        int n = cus[dev & 63].load(std::memory_order_relaxed);
        if (!n) {
            TRITD_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
            cus[dev & 63].store(n, std::memory_order_relaxed);
        }
        K5Args32 b = a;
        b.slots = (int64_t)n;  // one workgroup per CU per round of dispatch
        hipLaunchKernelGGL(k5_f32s<256>, dim3((unsigned)k5_parts32(g)), dim3(256), 0, st, b);
        TRITD_CHECK_LAUNCH();
        return;
    }
    const dim3 grid(k5_grid(g)), block(64 * K5W);
#define K5F_CASE(RPV)                                                        \
    case RPV:                                                                \
        if (prologue)                                                        \
            hipLaunchKernelGGL((k5_f32<RPV, true>), grid, block, 0, st, a);  \
        else                                                                 \
            hipLaunchKernelGGL((k5_f32<RPV, false>), grid, block, 0, st, a); \
        break;
    switch (g.RP) {
        K5F_CASE(16)
        K5F_CASE(32)
        K5F_CASE(48)
        K5F_CASE(64)
        K5F_CASE(128)
        K5F_CASE(256)
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by the fp32 K5");
    }
#undef K5F_CASE
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// layout conversions, norms, O rebuild, compact-E expansion, placement probe
// ---------------------------------------------------------------------------
// float offset of (i, j, t) in the fp32 tile-major layout
__host__ __device__ inline int64_t tm_offset32(int64_t i, int64_t j, int64_t t, int64_t n1p,
                                               int64_t ntt) {
    const int64_t g = (j * n1p + i) >> 4;
    const int l = (int)((((t & 15) >> 2) << 4) | (i & 15));
    return tm_tile_base(g, t >> 4, ntt) + 4 * l + (int)(t & 3);
}

__global__ __launch_bounds__(256) void k_to_tm32(const float* __restrict__ src, int64_t ld,
                                                 int64_t n1l, int64_t n2, int64_t n3, int64_t n1p,
                                                 int64_t ntt, int64_t Np, float* __restrict__ dst) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < Np; e += (int64_t)gridDim.x * 256) {
        const int64_t blk = e >> 8;  // ((g/4)*ntt + tt)*4 + g%4
        const int64_t q4 = blk >> 2, grp = q4 / ntt, tt = q4 - grp * ntt;
        const int64_t g = grp * 4 + (blk & 3);
        const int w = (int)(e & 255);
        const int l = w >> 2, r = w & 3;
        const int64_t t = 16 * tt + 4 * (l >> 4) + r;
        const int64_t row = 16 * g + (l & 15);
        const int64_t j = row / n1p, i = row - j * n1p;
        dst[e] = (i < n1l && j < n2 && t < n3) ? src[(t * n2 + j) * ld + i] : 0.0f;
    }
}

__global__ __launch_bounds__(256) void k_from_tm32(const float* __restrict__ src, int64_t n1l,
                                                   int64_t n2, int64_t n3, int64_t n1p, int64_t ntt,
                                                   float* __restrict__ dst, int64_t ld) {
    const int64_t total = n1l * n2 * n3;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * 256) {
        const int64_t i = e % n1l, jt = e / n1l;
        const int64_t j = jt % n2, t = jt / n2;
        dst[(t * n2 + j) * ld + i] = src[tm_offset32(i, j, t, n1p, ntt)];
    }
}

static unsigned grid_for32(int64_t n) {
    int64_t b = cdiv(n, 256);
    return (unsigned)(b > 16384 ? 16384 : (b < 1 ? 1 : b));
}

void launch_to_tm32(const Geom& g, const float* src, int64_t ld, float* dst, hipStream_t st) {
    hipLaunchKernelGGL(k_to_tm32, dim3(grid_for32(g.Ntm)), dim3(256), 0, st, src, ld, g.n1l, g.n2,
                       g.n3, g.n1p, g.ntt, g.Ntm, dst);
    TRITD_CHECK_LAUNCH();
}

void launch_from_tm32(const Geom& g, const float* src, float* dst, int64_t ld, hipStream_t st) {
    hipLaunchKernelGGL(k_from_tm32, dim3(grid_for32(g.n1l * g.n2 * g.n3)), dim3(256), 0, st, src,
                       g.n1l, g.n2, g.n3, g.n1p, g.ntt, dst, ld);
    TRITD_CHECK_LAUNCH();
}

// sum of squares in double (norm(D(:)) of a single D: the root is rounded to
// single by the caller)
__global__ __launch_bounds__(256) void k_sumsq32(const float* __restrict__ X, int64_t n,
                                                 double* partial) {
    double s = 0.0;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        const double x = (double)X[e];
        s = fma(x, x, s);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
        partial[2 * blockIdx.x + 1] = 0.0;
    }
}

void launch_sumsq32(const Geom& g, const float* X, double* partial, int nblocks, hipStream_t st) {
    hipLaunchKernelGGL(k_sumsq32, dim3(nblocks), dim3(256), 0, st, X, g.Ntm, partial);
    TRITD_CHECK_LAUNCH();
}

// O_k from T_{k+1} = (D - O_k) + invL_next Y_L (the loop never stores O):
// O = (D + invL_next Y_L) - T evaluated in double, rounded to single.  T is
// in the TX order of the same tile: element (t = 4(l>>4)+r, i = l&15) sits
// at TX lane ((i&3)<<4)|t, slot i>>2.
__global__ __launch_bounds__(256) void k_o_fixup32(const float* __restrict__ D,
                                                   const float* __restrict__ YL,
                                                   const float* __restrict__ T, float invL_next,
                                                   float* O, int64_t n) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        const int64_t base = e & ~(int64_t)255;
        const int w = (int)(e & 255);
        const int l = w >> 2, r = w & 3;
        const int t = 4 * (l >> 4) + r, ii = l & 15;
        const int tx = 4 * (((ii & 3) << 4) | t) + (ii >> 2);
        const double v = ((double)D[e] + (double)invL_next * (double)YL[e]) - (double)T[base + tx];
        O[e] = (float)v;
    }
}

void launch_o_fixup32(const Geom& g, const float* D, const float* YL, const float* T,
                      float invL_next, float* O, hipStream_t st) {
    hipLaunchKernelGGL(k_o_fixup32, dim3(grid_for32(g.Ntm)), dim3(256), 0, st, D, YL, T, invL_next,
                       O, g.Ntm);
    TRITD_CHECK_LAUNCH();
}

__global__ __launch_bounds__(256) void k_ce_expand32(const float* __restrict__ CE, float* E,
                                                     int64_t ntiles) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= ntiles) return;
    __shared__ __attribute__((aligned(16))) float cimg[4][CE32_IMG];
    float* img = cimg[threadIdx.x >> 6];
    for (int q = lane; q < CE32_IMG; q += 64) img[q] = 0.0f;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    float e[4];
    if (ce32_decode(CE[b * CE32_SLOT + lane], lane, img, e)) return;  // dense: E holds it
    reinterpret_cast<f4*>(E)[b * 64 + lane] = f4{e[0], e[1], e[2], e[3]};
}

void launch_ce_expand32(const Geom& g, const float* CE, float* E, hipStream_t st) {
    const int64_t ntiles = g.Ntm / 256;
    hipLaunchKernelGGL(k_ce_expand32, dim3((unsigned)cdiv(ntiles, 4)), dim3(256), 0, st, CE, E,
                       ntiles);
    TRITD_CHECK_LAUNCH();
}

// K5's fp32 HBM pattern without arithmetic (placement probing)
__global__ __launch_bounds__(256) void k_pool_probe32(float* D, float* YL, float* YO, float* T,
                                                      float* CE, int64_t tiles4, int64_t ntt) {
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= tiles4) return;
    f4* P[4] = {reinterpret_cast<f4*>(D), reinterpret_cast<f4*>(YL), reinterpret_cast<f4*>(YO),
                reinterpret_cast<f4*>(T)};
    struct R {
        f4 x[3];
        float ce;
    };
    auto tb = [&](int64_t tt) { return tm_tile_base(tile, tt, ntt); };
    auto load = [&](int64_t tt, R& n) {
        const int64_t o = (tb(tt) >> 2) + lane;
#pragma unroll
        for (int f = 0; f < 3; ++f) n.x[f] = P[f][o];
        n.ce = CE[(tb(tt) >> 8) * CE32_SLOT + lane];
    };
    auto body = [&](int64_t tt, R& c, R& n, bool pf) {
        if (pf) {
            load(tt + 1, n);
            __builtin_amdgcn_sched_barrier(0);
        }
        const int64_t o = (tb(tt) >> 2) + lane;
        P[1][o] = c.x[0] + c.x[1];
        P[2][o] = c.x[2] - c.x[1];
        P[3][o] = c.x[0] - c.x[2];
        CE[(tb(tt) >> 8) * CE32_SLOT + lane] = c.ce + 1.0f;
    };
    R xa, xb;
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

void launch_pool_probe32(const Geom& g, float* D, float* YL, float* YO, float* T, float* CE,
                         hipStream_t st) {
    hipLaunchKernelGGL(k_pool_probe32, dim3((unsigned)(g.tiles4 / 4)), dim3(256), 0, st, D, YL, YO,
                       T, CE, g.tiles4, g.ntt);
    TRITD_CHECK_LAUNCH();
}

__global__ __launch_bounds__(256) void k_widen(const float* __restrict__ x, int64_t n, double* y) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
        y[e] = (double)x[e];
}

void launch_widen(const float* x, int64_t n, double* y, hipStream_t st) {
    hipLaunchKernelGGL(k_widen, dim3(grid_for32(n)), dim3(256), 0, st, x, n, y);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
