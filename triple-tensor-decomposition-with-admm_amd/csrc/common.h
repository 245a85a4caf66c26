// Shared definitions for libtritd (MI355X / gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "tritd.h"

namespace tritd {

// Error carried from the point of failure to the C-ABI boundary, where it is
// turned into a tritd_status + thread-local message (api.cpp).
struct Error : std::runtime_error {
    tritd_status code;
    Error(tritd_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// A HIP call that must succeed.  A call that returns success but leaves the
// thread's last error set (hipGetLastError: sticky until read) is reported
// here, by name, instead of at the next launch check (TRITD_CHECK_LAUNCH
// reads that same state): with every HIP call of the library either checked
// here or made through hip_quiet, and each entry point clearing the state it
// inherits (api.cpp guarded), a launch check reports only its own launch.
#define TRITD_HIP(expr)                                                                      \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            throw ::tritd::Error(e_ == hipErrorOutOfMemory ? TRITD_ERR_NOMEM : TRITD_ERR_HIP, \
                                 std::string(#expr) + ": " + hipGetErrorString(e_));        \
        e_ = hipPeekAtLastError();                                                           \
        if (e_ != hipSuccess) {                                                              \
            (void)hipGetLastError();                                                         \
            throw ::tritd::Error(TRITD_ERR_HIP, std::string(#expr) +                         \
                                                    " returned success but left the last "   \
                                                    "error set: " + hipGetErrorString(e_));  \
        }                                                                                    \
    } while (0)

// A HIP call whose failure is deliberately ignored (destructors, cleanup
// after an error): it must not leave the thread's last error behind either.
inline void hip_quiet(hipError_t e) {
    if (e != hipSuccess) (void)hipGetLastError();
}

// a launch's error, named by the launching site
#define TRITD_STR2_(x) #x
#define TRITD_STR_(x) TRITD_STR2_(x)
#define TRITD_CHECK_LAUNCH()                                                                 \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ != hipSuccess)                                                                \
            throw ::tritd::Error(TRITD_ERR_HIP, std::string("kernel launch at " __FILE__ ":" \
                                                            TRITD_STR_(__LINE__) ": ") +     \
                                                    hipGetErrorString(e_));                  \
    } while (0)

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
__host__ __device__ inline int64_t cdiv(int64_t x, int64_t m) { return (x + m - 1) / m; }

// Padded rank R -> RP (multiple of 16, the f64 MFMA tile edge).  The kernels
// are instantiated for these RP values (r = 1..8).
inline int padded_rank(int R) { return (int)round_up(R, 16); }
inline bool rp_supported(int RP) { return RP == 16 || RP == 32 || RP == 48 || RP == 64; }

// Geometry of one shard in the device layout:
//   big tensors (D, O, E, Y_L, Y_O, T) are TILE-MAJOR ("TM"):
//     ij-tile g = (j*n1p + i)/16 (16 consecutive rows i of one fibre j),
//     t-tile tt = t/16; tile (g, tt) = 256 contiguous doubles, and the 4
//     ij-tiles of a group g/4 (the 4 waves of one K5 workgroup) are
//     interleaved per t-tile: tile (g, tt) at ((g/4*ntt + tt)*4 + g%4)*256, so
//     a workgroup reads or writes 8 KB contiguous per tensor per t-tile.
//     Inside a tile, element (r, l) of the f64 MFMA C/D fragment
//     (t%16 = (l>>4) + 4r, i%16 = l&15) sits at (r>>1)*128 + 2l + (r&1), so a
//     wave reads/writes a tile as two fully contiguous 1 KB dwordx4 sweeps and
//     walks its ij-tile's t-tiles as one contiguous stream.  Pads are zero.
//     T alone uses the transposed in-tile order "TX": slot (s, l), at
//     (s>>1)*128 + 2l + (s&1), holds (i%16 = 4s + (l>>4), t%16 = l&15) — the
//     B-operand order of the mode-3 MFMA (k_contract.hip, K2).
//   padded column-major ("PC") X[(t*n2 + j)*n1p + i] is used only at the
//     host boundary and by the primitives.
//   factors      Ah[i*RP+k], AhT[k*n1p+i], Bh[j*RP+k], Ch[t*RP+k], ChT[k*n3p+t]
//   W            Wk[k*plane + j*n1p + i] (plane = n1p*n2)
struct Geom {
    int64_t n1 = 0, n2 = 0, n3 = 0;  // global problem
    int64_t i0 = 0, i1 = 0;          // shard rows
    int64_t n1l = 0;                 // i1 - i0
    int64_t n1p = 0, n3p = 0;        // padded
    int r = 0, R = 0, RP = 0;
    int64_t plane = 0;               // n1p * n2
    int64_t Np = 0;                  // plane * n3p
    int64_t tiles = 0;               // plane / 16 (ij-tiles of 16 rows)
    int64_t ntt = 0;                 // n3p / 16 (t-tiles)
    int64_t tiles4 = 0;              // tiles rounded up to the group of 4
    int64_t Ntm = 0;                 // doubles of one tile-major tensor (tiles4*ntt*256)
    int tsplit = 1;                  // chunks of K5's t-walk (k5_tsplit, fixed at session creation)
};

inline Geom make_geom(int64_t n1, int64_t n2, int64_t n3, int64_t i0, int64_t i1, int r) {
    Geom g;
    g.n1 = n1; g.n2 = n2; g.n3 = n3; g.i0 = i0; g.i1 = i1; g.n1l = i1 - i0;
    g.n1p = round_up(g.n1l, 16);
    g.n3p = round_up(n3, 16);
    g.r = r; g.R = r * r; g.RP = padded_rank(g.R);
    g.plane = g.n1p * n2;
    g.Np = g.plane * g.n3p;
    g.tiles = g.plane / 16;
    g.ntt = g.n3p / 16;
    g.tiles4 = round_up(g.tiles, 4);
    g.Ntm = g.tiles4 * g.ntt * 256;
    return g;
}

// Scalars of one ADMM iteration, precomputed on the host from the
// deterministic mu schedule (triple_decomp_ADMM.m:16-17,56-57) so that every
// device expression uses the same IEEE scalars MATLAB would.
struct IterScalars {
    double muL, muO;
    double invL, invO;   // 1/muL, 1/muO          (:41,:42,:46)
    double thr;          // lambda/muO            (:47)
    double den;          // muL + muO             (:43)
    double invL_next;    // 1/muL of the next iteration (fused T formation, :33)
    double muO_prev;     // muO of the previous iteration (derived Y_O, k_admm.hip)
    double rden;         // 1/den, correctly rounded (K5's division by den, k_admm.hip)
    double cprev;        // invO * muO_prev (K5's R1 + R2 and R3 through E^(k) - E^(k-1), k_admm.hip)
};

// first double of tile (g, tt) in the tile-major layout
// Compact E (CE).  E is the soft-thresholded outlier tensor, mostly zeros
// (<= 5 % nonzero and <= 33 per 256-element tile on the bench workload), so
// it is kept as one 32-double slot per tile (slot of tile ordinal b =
// tm_tile_base(g, tt)/256 at CE + 32 b):
//   words 0..26:  the nonzero values, ordered by (w, l) (see below)
//   bytes CE_IDX_BYTE + q (words 27..30): the in-tile position of value q,
//                 64 w + l for the element lane l holds as MFMA C/D register
//                 element (p, q) = (w >> 1, w & 1), i.e. the TM in-tile
//                 position 128 p + 2 l + q
//   word 31:      the count in its low dword (all ones: dense)
// A tile with more than CE_CAP nonzeros is stored densely in E (TM) and its
// count is all ones.  Zeros are stored as +0 (MATLAB's E may hold -0, which is
// numerically identical in every later use).  Decoding scatters the values
// into a per-wave LDS tile image of CE_IMG doubles (256 + a junk word per lane).
constexpr int CE_SLOT = 32;
constexpr int CE_CAP = 27;
constexpr int CE_IDX_BYTE = 8 * CE_CAP;  // 216
constexpr int CE_CNT_WORD = 31;
constexpr int CE_IMG = 256 + 64;

__host__ __device__ inline int64_t tm_tile_base(int64_t g, int64_t tt, int64_t ntt) {
    return ((((g >> 2) * ntt + tt) << 2) + (g & 3)) << 8;
}

// TM offset of element (i, j, t) of a shard (i < n1p, t < n3p)
__host__ __device__ inline int64_t tm_offset(int64_t i, int64_t j, int64_t t, int64_t n1p, int64_t ntt) {
    const int64_t g = (j * n1p + i) >> 4;
    const int il = (int)(i & 15), tl = (int)(t & 15);
    const int r = tl >> 2, l = ((tl & 3) << 4) | il;
    return tm_tile_base(g, t >> 4, ntt) + ((r >> 1) << 7) + (l << 1) + (r & 1);
}

}  // namespace tritd
