// Times the R x R solves alone (back-to-back launches on one stream):
// k_solve (Gauss-Jordan sweep) cold, and k_solve_ns warm-started from the
// inverse of a perturbed Gram (relative perturbation eps: ||E0|| ~ eps*cond),
// and checks inv(G)*G = I.
// build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Iinclude -I<csrc> tools/solve_ns_bench.hip -o tools/solve_ns_bench
#include "../triple-tensor-decomposition-with-admm_amd/csrc/k_contract.hip"
#include <cstdio>
#include <vector>
#include <cmath>
#include <cstdlib>
using namespace tritd;
int main(int argc, char** argv) {
    constexpr int RP = 64;
    const int R = 64;
    std::vector<double> P(RP * RP), Q(RP * RP), P2(RP * RP);
    std::vector<double> X(400 * RP);
    unsigned s = 1;
    for (auto& x : X) { s = s * 1103515245u + 12345u; x = ((s >> 8) & 0xffff) / 65536.0 - 0.5; }
    for (int i = 0; i < RP; ++i) for (int j = 0; j < RP; ++j) {
        double a = 0; for (int r = 0; r < 400; ++r) a += X[r * RP + i] * X[r * RP + j];
        P[i * RP + j] = a; Q[i * RP + j] = 1.0 + 0.01 * ((i * 7 + j * 7) % 5);
    }
    double *dP, *dP2, *dQ, *dG; int *flags, *stop;
    hipMalloc(&dP, 8 * RP * RP); hipMalloc(&dP2, 8 * RP * RP); hipMalloc(&dQ, 8 * RP * RP); hipMalloc(&dG, 8 * RP * RP);
    hipMalloc(&flags, 4); hipMalloc(&stop, 4); hipMemset(flags, 0, 4); hipMemset(stop, 0, 4);
    hipMemcpy(dP, P.data(), 8 * RP * RP, hipMemcpyHostToDevice);
    hipMemcpy(dQ, Q.data(), 8 * RP * RP, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto check = [&](const char* what, float us) {
        std::vector<double> G(RP * RP);
        hipMemcpy(G.data(), dG, 8 * RP * RP, hipMemcpyDeviceToHost);
        double err = 0;
        for (int i = 0; i < R; ++i) for (int j = 0; j < R; ++j) {
            double a = 0; for (int k = 0; k < R; ++k) a += G[i * RP + k] * (P[k * RP + j] * Q[k * RP + j] + (k == j ? 1e-3 : 0));
            err = fmax(err, fabs(a - (i == j)));
        }
        int fl = 0; hipMemcpy(&fl, flags, 4, hipMemcpyDeviceToHost);
        printf("%-34s %8.2f us/solve  max|inv*G-I| %.2e  flag %d\n", what, us, err, fl);
    };
    const int N = 100;
    // GJ sweep, cold
    hipLaunchKernelGGL(k_solve<RP>, dim3(1), dim3(RP * 64 / SOLVE_ROWS), 0, 0, dP, dQ, R, 1e-3, dG, flags, stop);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int k = 0; k < N; ++k)
        hipLaunchKernelGGL(k_solve<RP>, dim3(1), dim3(RP * 64 / SOLVE_ROWS), 0, 0, dP, dQ, R, 1e-3, dG, flags, stop);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    check("k_solve (sweep)", ms * 1000 / N);
    // NS cold (zero start -> sweep fallback)
    hipEventRecord(e0);
    for (int k = 0; k < N; ++k) {
        hipMemsetAsync(dG, 0, 8 * RP * RP, 0);
        hipLaunchKernelGGL(k_solve_ns<RP>, dim3(1), dim3(RP * 16), 0, 0, dP, dQ, R, 1e-3, dG, flags, stop);
    }
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    check("k_solve_ns cold (+memset)", ms * 1000 / N);
    for (double eps : {1e-2, 1e-4, 1e-6, 1e-9, 0.0}) {
        for (int i = 0; i < RP * RP; ++i) { s = s * 1103515245u + 12345u; P2[i] = P[i] * (1.0 + eps * (((s >> 8) & 0xffff) / 65536.0 - 0.5)); }
        for (int i = 0; i < RP; ++i) for (int j = 0; j < i; ++j) P2[i * RP + j] = P2[j * RP + i];
        hipMemcpy(dP2, P2.data(), 8 * RP * RP, hipMemcpyHostToDevice);
        // per launch: reset the start to inv(perturbed) by a sweep, then time NS alone via events
        float tot = 0;
        for (int k = 0; k < N; ++k) {
            hipLaunchKernelGGL(k_solve<RP>, dim3(1), dim3(RP * 64 / SOLVE_ROWS), 0, 0, dP2, dQ, R, 1e-3, dG, flags, stop);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_solve_ns<RP>, dim3(1), dim3(RP * 16), 0, 0, dP, dQ, R, 1e-3, dG, flags, stop);
            hipEventRecord(e1); hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1); tot += ms;
        }
        char buf[64]; snprintf(buf, sizeof buf, "k_solve_ns warm, perturb %.0e", eps);
        check(buf, tot * 1000 / N);
    }
    return 0;
}
