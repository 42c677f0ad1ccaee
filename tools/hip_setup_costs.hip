// Diagnostic: first-call costs of the HIP runtime operations a cold tray_render
// performs (device properties, stream creation, allocations, first launch).
//   hipcc --offload-arch=gfx950 -O2 tools/hip_setup_costs.hip -o tools/hip_setup_costs
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

__global__ void noop(int* p) {
    if (p && threadIdx.x == 1024) *p = 0;
}

int main() {
    auto t0 = std::chrono::steady_clock::now();
    int n = 0;
    (void)hipGetDeviceCount(&n);
    printf("{\"hipGetDeviceCount_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    printf(", \"hipGetDeviceProperties_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    (void)hipGetDeviceProperties(&prop, 0);
    printf(", \"hipGetDeviceProperties_again_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf(", \"hipDeviceGetAttribute_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    hipStream_t s1, s2;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    printf(", \"hipStreamCreate_first_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    printf(", \"hipStreamCreate_second_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    void* big = nullptr;
    (void)hipMalloc(&big, (size_t)1415577600);
    printf(", \"hipMalloc_1p4GB_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    void* small = nullptr;
    (void)hipMalloc(&small, (size_t)3686400);
    printf(", \"hipMalloc_3p7MB_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s1, (int*)nullptr);
    (void)hipStreamSynchronize(s1);
    printf(", \"first_launch_s1_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s2, (int*)nullptr);
    (void)hipStreamSynchronize(s2);
    printf(", \"first_launch_s2_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, hipStreamPerThread, (int*)nullptr);
    (void)hipStreamSynchronize(hipStreamPerThread);
    printf(", \"first_launch_per_thread_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s1, (int*)nullptr);
    (void)hipStreamSynchronize(s1);
    printf(", \"second_launch_s1_ms\": %.3f", ms_since(t0));
    static char host[3686400];
    t0 = std::chrono::steady_clock::now();
    (void)hipMemcpyAsync(host, small, sizeof(host), hipMemcpyDeviceToHost, s1);
    (void)hipStreamSynchronize(s1);
    printf(", \"d2h_pageable_first_ms\": %.3f", ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    (void)hipMemcpyAsync(host, small, sizeof(host), hipMemcpyDeviceToHost, s1);
    (void)hipStreamSynchronize(s1);
    printf(", \"d2h_pageable_second_ms\": %.3f}\n", ms_since(t0));
    return 0;
}
