// Store-data hazard probe for gfx950 (MI355X).  A wide VMEM store
// (buffer_store_dwordx4) is followed, K wait states later, by an instruction
// that rewrites the first 64 bits of its data registers; every lane then
// checks in memory that the store wrote the ORIGINAL data.  Many waves store
// at once (the memory pipeline under load, as in K5).  A diagnostic for the
// dense-E K5 corruption of round 4.
//
//   hipcc --offload-arch=gfx950 -O2 tools/store_hazard.hip -o /tmp/store_hazard
//   /tmp/store_hazard
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

constexpr int ITERS = 64;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, bytes, 0x00020000);
}

// OP 0: v_mov_b64 (64-bit VALU) over the low 64 bits of the data
// OP 1: v_mov_b32 over the low dword
// OP 2: v_add_f64 over the low 64 bits
// OP 3: nothing (control)
// AUX 2: the store carries the nontemporal bit (as K5's streams)
// PRE: the instructions that produce the data right before the store
// (PRE_NOP: with a pad; PRE_DP: a DP fma writes the last pair with no pad,
// as the compiler emits K5's Y_L stores)
#define PRE_NOP "v_mov_b64 v[20:21], %[a]\nv_mov_b64 v[22:23], %[b]\ns_nop 4\n"
#define PRE_DP "v_mov_b64 v[20:21], %[a]\nv_mov_b64 v[22:23], %[b]\ns_nop 4\nv_fma_f64 v[22:23], %[b], 1.0, 0\n"
#define FILL_NOP ".rept %[k]\n v_nop\n .endr\n"
// K independent DP adds (alternating registers) / K dependent DP adds
#define FILL_DPI ".rept %[k]\n v_add_f64 v[30:31], %[j], 1.0\n v_add_f64 v[32:33], %[j], 1.0\n .endr\n"
#define FILL_DPD ".rept %[k]\n v_add_f64 v[30:31], v[30:31], 1.0\n .endr\n"
#define FILL_DPR ".rept %[k]\n v_fma_f64 v[30:31], v[20:21], 1.0, 0\n .endr\n"
#define PRE_MF "v_mfma_f64_16x16x4_f64 v[40:47], %[a], %[b], v[40:47]\n" \
               "v_mfma_f64_16x16x4_f64 v[40:47], %[a], %[b], v[40:47]\n" \
               "v_mfma_f64_16x16x4_f64 v[40:47], %[a], %[b], v[40:47]\n" \
               "v_mfma_f64_16x16x4_f64 v[40:47], %[a], %[b], v[40:47]\n" \
               "v_mfma_f64_16x16x4_f64 v[40:47], %[a], %[b], v[40:47]\n" \
               "v_mfma_f64_16x16x4_f64 v[40:47], %[a], %[b], v[40:47]\n" \
               "v_fma_f64 v[20:21], %[a], 1.0, 0\nv_fma_f64 v[22:23], %[b], 1.0, 0\n"
// loads in flight ahead of the store (as K5's prefetch of tile tt+1)
#define PRE_LD "buffer_load_dwordx4 v[48:51], %[vo], %[rl], %[so] offen nt\n" \
               "buffer_load_dwordx4 v[52:55], %[vo], %[rl], %[so] offen offset:1024 nt\n" \
               "buffer_load_dwordx4 v[56:59], %[vo], %[rl], %[so] offen offset:2048 nt\n" \
               "buffer_load_dwordx4 v[60:63], %[vo], %[rl], %[so] offen offset:3072 nt\n" \
               "v_fma_f64 v[20:21], %[a], 1.0, 0\nv_fma_f64 v[22:23], %[b], 1.0, 0\n"
#define FILL FILL_NOP
#define PROBE_ASM(NT, OVER) PROBE_ASM_ST("buffer_store_dwordx4 v[20:23], %[vo], %[rs], %[so] offen" NT "\n", OVER)
// ST: the store itself (SGPR soffset as K5's streams, a constant soffset —
// the case LLVM pads — or a global store)
#define ST_SGPR "buffer_store_dwordx4 v[20:23], %[vo], %[rs], %[so] offen nt\n"
#define ST_CONST "buffer_store_dwordx4 v[20:23], %[vt], %[rs], 0 offen nt\n"
#define ST_GLOBAL "global_store_dwordx4 %[ga], v[20:23], off nt\n"
#define PROBE_ASM_ST(STORE, OVER)                                                            \
    asm volatile("" PRE                                                                      \
                 STORE                                                                      \
                 FILL OVER                                                                  \
                 :                                                                          \
                 : [a] "v"(a), [b] "v"(b), [j] "v"(junk), [vo] "v"(voff), [rs] "s"(r),     \
                   [so] "s"(soff), [k] "i"(K), [la] "v"(laddr), [ro] "s"(rj), [rl] "s"(rld),  \
                   [ga] "v"(gaddr + it * 128), [vt] "v"(voff + it * 1024)                                                     \
                 : "v20", "v21", "v22", "v23", "v30", "v31", "v32", "v33", "v40", "v41", "v42", "v43", \
                   "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
                   "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "memory")
template <int K, int OP, int AUX, int DP, int FL>
__global__ __launch_bounds__(256) void probe(double* out) {
    const int tid = blockIdx.x * 256 + threadIdx.x;
    // each wave stores ITERS tiles of 1 KB; lane l at 16 l
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = threadIdx.x & 63;
    double* base = out + (size_t)wave * ITERS * 128;
    const __amdgpu_buffer_rsrc_t r = rsrc_of(base, ITERS * 1024);
    const int voff = lane * 16;
    // ST_CONST / ST_GLOBAL: the tile offset goes into the address instead
    double* gaddr = base + 2 * lane;
    // an LDS word and a global word holding junk, read back into the data
    // registers of the in-flight store (OP 4 / OP 5)
    __shared__ double lj[64];
    lj[lane] = 1e300;
    __syncthreads();
    const int laddr = (int)(size_t)&lj[lane];
    const __amdgpu_buffer_rsrc_t rj = rsrc_of(out + (size_t)gridDim.x * 4 * ITERS * 128, 1024);
    // a source the loads stream from (the second half of the allocation)
    const __amdgpu_buffer_rsrc_t rld = rsrc_of(out + (size_t)gridDim.x * 4 * ITERS * 128 + 128 +
                                                   (size_t)wave * ITERS * 512, ITERS * 4096);
    asm volatile("v_mov_b64 v[40:41], 0\nv_mov_b64 v[42:43], 0\nv_mov_b64 v[44:45], 0\nv_mov_b64 v[46:47], 0\ns_nop 4\n" ::
                     : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    for (int it = 0; it < ITERS; ++it) {
        const double a = (double)(tid * ITERS + it) + 0.25, b = -a;
        const double junk = 1e300;
        const int soff = __builtin_amdgcn_readfirstlane(it * 1024);
#define PRE PRE_NOP
        if constexpr (FL > 0) {
#undef PRE
#define PRE PRE_DP
#undef FILL
#define FILL FILL_DPI
            if constexpr (FL == 1) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\n");
#undef FILL
#define FILL FILL_DPD
            if constexpr (FL == 2) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\n");
#undef FILL
#define FILL FILL_DPR
            if constexpr (FL == 3) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\n");
#undef PRE
#define PRE PRE_MF
#undef FILL
#define FILL FILL_NOP
            if constexpr (FL == 4) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\n");
#undef FILL
#define FILL FILL_DPI
            if constexpr (FL == 5) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\n");
#undef PRE
#define PRE PRE_LD
#undef FILL
#define FILL FILL_NOP
            if constexpr (FL == 6) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\ns_waitcnt vmcnt(0)\n");
#undef FILL
#define FILL FILL_DPI
            if constexpr (FL == 7) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\ns_waitcnt vmcnt(0)\n");
#undef FILL
#define FILL FILL_NOP
#undef PRE
#define PRE PRE_NOP
        } else if constexpr (DP) {
#undef PRE
#define PRE PRE_DP
            if constexpr (OP == 0) PROBE_ASM(" nt", "v_mov_b64 v[20:21], %[j]\n");
            if constexpr (OP == 1) PROBE_ASM(" nt", "v_mov_b32 v20, 0\n");
            if constexpr (OP == 2) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\n");
            if constexpr (OP == 3) PROBE_ASM(" nt", "");
            if constexpr (OP == 4) PROBE_ASM(" nt", "ds_read_b64 v[20:21], %[la]\ns_waitcnt lgkmcnt(0)\n");
            if constexpr (OP == 5) PROBE_ASM(" nt", "buffer_load_dwordx2 v[20:21], %[vo], %[ro], 0 offen\ns_waitcnt vmcnt(0)\n");
            // round 5: the compiler's own K5 sequences (k_admm.hip built with
            // TRITD_STORE_KEEP=0: a 64-bit VALU write of the first data pair
            // right behind a buffer_store_dwordx4 with an SGPR soffset)
            if constexpr (OP == 6) PROBE_ASM(" nt", "v_lshl_add_u64 v[20:21], %[j], 0, %[j]\n");
            if constexpr (OP == 7) PROBE_ASM(" nt", "v_add_f64 v[22:23], %[j], %[j]\n");  // the second pair
            if constexpr (OP == 8) PROBE_ASM_ST(ST_CONST, "v_add_f64 v[20:21], %[j], %[j]\n");
            if constexpr (OP == 9) PROBE_ASM_ST(ST_GLOBAL, "v_add_f64 v[20:21], %[j], %[j]\n");
            if constexpr (OP == 10) PROBE_ASM_ST(ST_SGPR, "v_fma_f64 v[20:21], %[j], %[j], %[j]\n");
#undef PRE
#define PRE PRE_NOP
        } else if constexpr (AUX == 2) {
            if constexpr (OP == 0) PROBE_ASM(" nt", "v_mov_b64 v[20:21], %[j]\n");
            if constexpr (OP == 1) PROBE_ASM(" nt", "v_mov_b32 v20, 0\n");
            if constexpr (OP == 2) PROBE_ASM(" nt", "v_add_f64 v[20:21], %[j], %[j]\n");
            if constexpr (OP == 3) PROBE_ASM(" nt", "");
        } else {
            if constexpr (OP == 0) PROBE_ASM("", "v_mov_b64 v[20:21], %[j]\n");
            if constexpr (OP == 1) PROBE_ASM("", "v_mov_b32 v20, 0\n");
            if constexpr (OP == 2) PROBE_ASM("", "v_add_f64 v[20:21], %[j], %[j]\n");
            if constexpr (OP == 3) PROBE_ASM("", "");
        }
    }
}

template <int K, int OP, int AUX, int DP = 0, int FL = 0>
void run(double* d, std::vector<double>& h, int blocks, const char* name) {
    const size_t n = (size_t)blocks * 4 * ITERS * 128;
    CHECK(hipMemset(d, 0, n * sizeof(double)));
    hipLaunchKernelGGL((probe<K, OP, AUX, DP, FL>), dim3(blocks), dim3(256), 0, 0, d);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost));
    long bad = 0, bad_lane[16] = {0}, bad_w[2] = {0, 0};
    for (int wave = 0; wave < blocks * 4; ++wave)
        for (int it = 0; it < ITERS; ++it)
            for (int lane = 0; lane < 64; ++lane) {
                const int tid = wave * 64 + lane;
                const double a = (double)(tid * ITERS + it) + 0.25;
                const double* p = &h[((size_t)wave * ITERS + it) * 128 + 2 * lane];
                if (p[0] != a || p[1] != -a) {
                    ++bad;
                    bad_w[0] += p[0] != a;
                    bad_w[1] += p[1] != -a;
                    ++bad_lane[lane & 15];
                }
            }
    std::printf("%-28s K=%2d aux=%d dp=%d fl=%d  wrong %ld of %zu", name, K, AUX, DP, FL, bad, n / 2);
    if (bad) {
        std::printf("  words %ld/%ld  by lane%%16:", bad_w[0], bad_w[1]);
        for (int l = 0; l < 16; ++l) std::printf(" %ld", bad_lane[l]);
    }
    std::printf("\n");
}

int main() {
    const int blocks = 4096;
    const size_t n = (size_t)blocks * 4 * ITERS * 128;
    double* d;
    CHECK(hipMalloc(&d, 5 * n * sizeof(double) + 2048));
    {
        std::vector<double> junk(128, 1e300);
        CHECK(hipMemcpy(d + n, junk.data(), 1024, hipMemcpyHostToDevice));
    }
    std::vector<double> h(n);
    run<0, 3, 0>(d, h, blocks, "control");
    // round 5: the writers the compiler placed behind K5's stores
    run<0, 2, 2, 1>(d, h, blocks, "sgpr soff, v_add_f64");
    run<1, 2, 2, 1>(d, h, blocks, "sgpr soff, v_add_f64");
    run<0, 6, 2, 1>(d, h, blocks, "sgpr soff, v_lshl_add_u64");
    run<1, 6, 2, 1>(d, h, blocks, "sgpr soff, v_lshl_add_u64");
    run<0, 10, 2, 1>(d, h, blocks, "sgpr soff, v_fma_f64");
    run<1, 10, 2, 1>(d, h, blocks, "sgpr soff, v_fma_f64");
    run<0, 7, 2, 1>(d, h, blocks, "sgpr soff, 2nd pair add");
    run<1, 7, 2, 1>(d, h, blocks, "sgpr soff, 2nd pair add");
    // the store forms the compiler pads (one wait state)
    run<0, 8, 2, 1>(d, h, blocks, "const soff, v_add_f64");
    run<1, 8, 2, 1>(d, h, blocks, "const soff, v_add_f64");
    // round 6: the scan window of tests/test_isa_store_war.py
    // is two wait states; the constant-soffset form still lost 16 lanes at one,
    // so it is measured at two and three, three times each
    for (int rep = 0; rep < 3; ++rep) {
        run<1, 8, 2, 1>(d, h, blocks, "const soff, v_add_f64");
        run<2, 8, 2, 1>(d, h, blocks, "const soff, v_add_f64");
        run<3, 8, 2, 1>(d, h, blocks, "const soff, v_add_f64");
        run<2, 2, 2, 1>(d, h, blocks, "sgpr soff, v_add_f64");
        run<2, 6, 2, 1>(d, h, blocks, "sgpr soff, v_lshl_add_u64");
    }
    run<0, 9, 2, 1>(d, h, blocks, "global, v_add_f64");
    run<1, 9, 2, 1>(d, h, blocks, "global, v_add_f64");
    CHECK(hipFree(d));
    return 0;
}
