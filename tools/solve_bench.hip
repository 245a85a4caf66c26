// Times k_solve<64> alone (back-to-back launches) and checks inv(G)*G = I.
// Built in variants by tools/solve_bench.sh (-DSOLVE_ROWS_OVERRIDE, -DSOLVE_RCP).
#include "../triple-tensor-decomposition-with-admm_amd/csrc/k_contract.hip"
#include <cstdio>
#include <vector>
#include <cmath>
#include <cstdlib>
int main(int argc, char** argv) {
    const int RP = argc > 1 ? atoi(argv[1]) : 64, R = argc > 2 ? atoi(argv[2]) : RP;
    std::vector<double> P(RP * RP), Q(RP * RP);
    // SPD Grams: X^T X of random 200 x 64
    std::vector<double> X(400 * RP);
    unsigned s = 1;
    for (auto& x : X) { s = s * 1103515245u + 12345u; x = ((s >> 8) & 0xffff) / 65536.0 - 0.5; }
    for (int i = 0; i < RP; ++i) for (int j = 0; j < RP; ++j) {
        double a = 0; for (int r = 0; r < 400; ++r) a += X[r * RP + i] * X[r * RP + j];
        P[i * RP + j] = a; Q[i * RP + j] = 1.0 + 0.01 * ((i * 7 + j * 7) % 5);  // symmetric
    }
    double *dP, *dQ, *dG; int *flags, *stop;
    hipMalloc(&dP, 8 * RP * RP); hipMalloc(&dQ, 8 * RP * RP); hipMalloc(&dG, 8 * RP * RP);
    hipMalloc(&flags, 4); hipMalloc(&stop, 4); hipMemset(flags, 0, 4); hipMemset(stop, 0, 4);
    hipMemcpy(dP, P.data(), 8 * RP * RP, hipMemcpyHostToDevice);
    hipMemcpy(dQ, Q.data(), 8 * RP * RP, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    tritd::launch_solve(RP, R, dP, dQ, 1e-3, dG, flags, stop, 0);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int k = 0; k < 200; ++k) tritd::launch_solve(RP, R, dP, dQ, 1e-3, dG, flags, stop, 0);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<double> G(RP * RP);
    hipMemcpy(G.data(), dG, 8 * RP * RP, hipMemcpyDeviceToHost);
    double err = 0;
    for (int i = 0; i < R; ++i) for (int j = 0; j < R; ++j) {
        double a = 0; for (int k = 0; k < R; ++k) a += G[i * RP + k] * (P[k * RP + j] * Q[k * RP + j] + (k == j ? 1e-3 : 0));
        err = fmax(err, fabs(a - (i == j)));
    }
    int fl = 0;
    hipMemcpy(&fl, flags, 4, hipMemcpyDeviceToHost);
    printf("%s RP=%d R=%d: %.2f us/solve  max|inv*G-I| %.2e  flag %d\n", VARIANT, RP, R, ms * 1000 / 200, err, fl);
    return 0;
}
