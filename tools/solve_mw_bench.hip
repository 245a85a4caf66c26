// Times launch_solve at RP = 128 / 256 (k_solve_mw by default; TRITD_SOLVE=big
// for the one-workgroup kernels) back to back, and checks max|inv(G)*G - I|.
// usage: solve_mw_bench RP R
#include "../triple-tensor-decomposition-with-admm_amd/csrc/k_contract.hip"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
int main(int argc, char** argv) {
    const int RP = argc > 1 ? atoi(argv[1]) : 256, R = argc > 2 ? atoi(argv[2]) : RP;
    std::vector<double> P(RP * RP, 0.0), Q(RP * RP, 0.0);
    const int NR = 3 * RP;  // SPD Gram X^T X of a random NR x R
    std::vector<double> X((size_t)NR * R);
    unsigned s = 1;
    for (auto& x : X) { s = s * 1103515245u + 12345u; x = ((s >> 8) & 0xffff) / 65536.0 - 0.5; }
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < R; ++j) {
            double a = 0;
            for (int r = 0; r < NR; ++r) a += X[(size_t)r * R + i] * X[(size_t)r * R + j];
            P[i * RP + j] = a;
            Q[i * RP + j] = 1.0 + 0.01 * ((i * 7 + j * 7) % 5);
        }
    const size_t gn = tritd::ginv_count(RP);
    double *dP, *dQ, *dG;
    int *flags, *stop;
    hipMalloc(&dP, 8 * RP * RP); hipMalloc(&dQ, 8 * RP * RP); hipMalloc(&dG, 8 * gn);
    hipMemset(dG, 0, 8 * gn);
    hipMalloc(&flags, 4); hipMalloc(&stop, 4); hipMemset(flags, 0, 4); hipMemset(stop, 0, 4);
    hipMemcpy(dP, P.data(), 8 * RP * RP, hipMemcpyHostToDevice);
    hipMemcpy(dQ, Q.data(), 8 * RP * RP, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    tritd::launch_solve(RP, R, dP, dQ, 1e-3, dG, flags, stop, 0);
    hipDeviceSynchronize();
    const int N = 50;
    hipEventRecord(e0);
    for (int k = 0; k < N; ++k) tritd::launch_solve(RP, R, dP, dQ, 1e-3, dG, flags, stop, 0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<double> G(RP * RP);
    hipMemcpy(G.data(), dG, 8 * RP * RP, hipMemcpyDeviceToHost);
    double err = 0, pad = 0;
    for (int i = 0; i < RP; ++i)
        for (int j = 0; j < RP; ++j) {
            if (i >= R || j >= R) { pad = fmax(pad, fabs(G[i * RP + j])); continue; }
            double a = 0;
            for (int k = 0; k < R; ++k) a += G[i * RP + k] * (P[k * RP + j] * Q[k * RP + j] + (k == j ? 1e-3 : 0));
            err = fmax(err, fabs(a - (i == j)));
        }
    int fl = 0;
    hipMemcpy(&fl, flags, 4, hipMemcpyDeviceToHost);
    // a stopped launch must leave the inverse alone and not hang
    hipMemset(stop, 0xff, 4);
    for (int k = 0; k < 3; ++k) tritd::launch_solve(RP, R, dP, dQ, 1e-3, dG, flags, stop, 0);
    hipError_t st = hipDeviceSynchronize();
    const char* v = getenv("TRITD_SOLVE");
    printf("solve[%s] RP=%d R=%d: %.2f us/solve  max|inv*G-I| %.2e  pad %.1e  flags %d  stopped-launch %s\n",
           v ? v : "default", RP, R, ms * 1000 / N, err, pad, fl, st == hipSuccess ? "ok" : "ERR");
    return 0;
}
