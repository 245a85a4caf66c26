// Cost of cross-stream synchronisation on the critical (main) stream:
// a chain of 40 small dependent kernels on stream A, with after each kernel
//   none          nothing
//   event         hipEventRecord(A) + hipStreamWaitEvent(B)  (B runs a tiny kernel)
//   writevalue    hipStreamWriteValue32(A) + hipStreamWaitValue32(B)
// Reports the chain's wall time per link (device time, events around the chain).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
__global__ void k_small(double* p, int n) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = p[i] * 1.0000001 + 1.0;
}
int main() {
    double *a, *b; unsigned* flag;
    const int n = 64 * 256;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8)); CK(hipMalloc(&flag, 4096));
    CK(hipMemset(a, 0, n * 8)); CK(hipMemset(b, 0, n * 8)); CK(hipMemset(flag, 0, 4096));
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    int lo, hi; CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, hi));
    hipEvent_t t0, t1, ev[64];
    CK(hipEventCreate(&t0)); CK(hipEventCreate(&t1));
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const int L = 40;
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, A));
            for (int q = 0; q < L; ++q) {
                hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, A, a, n);
                if (mode == 1) {
                    CK(hipEventRecord(ev[q], A));
                    CK(hipStreamWaitEvent(B, ev[q], 0));
                    hipLaunchKernelGGL(k_small, dim3(1), dim3(256), 0, B, b, 256);
                } else if (mode == 2) {
                    CK(hipStreamWriteValue32(A, flag + q, 1, 0));
                    CK(hipStreamWaitValue32(B, flag + q, 1, hipStreamWaitValueGte, 0xffffffffu));
                    hipLaunchKernelGGL(k_small, dim3(1), dim3(256), 0, B, b, 256);
                } else if (mode == 3) {  // B -> A direction: A waits on B's tiny kernel
                    hipLaunchKernelGGL(k_small, dim3(1), dim3(256), 0, B, b, 256);
                    CK(hipEventRecord(ev[q], B));
                    CK(hipStreamWaitEvent(A, ev[q], 0));
                }
            }
            CK(hipEventRecord(t1, A));
            CK(hipEventSynchronize(t1));
            CK(hipStreamSynchronize(B));
            float ms; CK(hipEventElapsedTime(&ms, t0, t1));
            if (mode == 2) CK(hipMemset(flag, 0, 4096));
            printf("mode %-11s rep %d: %.2f us per link\n",
                   mode == 0 ? "none" : mode == 1 ? "event" : mode == 2 ? "writevalue" : "event(B->A)", rep, ms * 1000 / L);
        }
    }
    return 0;
}
