// Same-address vs spread global atomics on MI355X (experiment, not product):
// G workgroups x A atomics each, returning (the value used) or not, on one
// counter / one counter per 64 workgroups / one per workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_atomic(int* c, int spread, int per, int ret, int* sink) {
    int acc = 0;
    if (threadIdx.x == 0) {
        int* p = c + (spread == 0 ? 0 : spread == 1 ? (blockIdx.x / 64) * 32 : blockIdx.x * 32);
        for (int a = 0; a < per; ++a) {
            if (ret) acc += atomicAdd(p, 1);
            else atomicAdd(p, 1);
        }
        if (ret && acc == -1) sink[0] = acc;
    }
}

int main() {
    int *c, *sink;
    hipMalloc(&c, 1 << 24);
    hipMalloc(&sink, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int G : {256, 2048, 8192})
        for (int per : {1, 8})
            for (int spread : {0, 1, 2})
                for (int ret : {0, 1}) {
                    hipMemset(c, 0, 1 << 24);
                    hipLaunchKernelGGL(k_atomic, dim3(G), dim3(256), 0, 0, c, spread, per, ret, sink);
                    hipDeviceSynchronize();
                    float best = 1e9;
                    for (int it = 0; it < 5; ++it) {
                        hipEventRecord(e0);
                        hipLaunchKernelGGL(k_atomic, dim3(G), dim3(256), 0, 0, c, spread, per, ret, sink);
                        hipEventRecord(e1);
                        hipEventSynchronize(e1);
                        float ms;
                        hipEventElapsedTime(&ms, e0, e1);
                        best = ms < best ? ms : best;
                    }
                    printf("G %5d per %d spread %d ret %d: %8.1f us  (%.1f ns per atomic)\n", G, per, spread, ret,
                           best * 1e3, best * 1e6 / (G * per));
                }
    return 0;
}
