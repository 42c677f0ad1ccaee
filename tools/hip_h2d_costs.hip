// Diagnostic: first-call costs of pageable host-to-device copies by size (the
// scene upload's hipMemcpy), after a tiny copy has warmed the runtime.
//   hipcc --offload-arch=gfx950 -O2 tools/hip_h2d_costs.hip -o tools/hip_h2d_costs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    void* dev = nullptr;
    (void)hipMalloc(&dev, (size_t)64 << 20);
    char* host = (char*)malloc((size_t)64 << 20);
    for (size_t i = 0; i < ((size_t)64 << 20); ++i) host[i] = (char)i;
    const size_t sizes[] = {256, 2048, 16384, 65536, 131072, 262144, 1 << 20, 4 << 20, 16 << 20};
    printf("[");
    for (int rep = 0; rep < 2; ++rep)
        for (size_t k = 0; k < sizeof(sizes) / sizeof(sizes[0]); ++k) {
            auto t0 = std::chrono::steady_clock::now();
            (void)hipMemcpy(dev, host, sizes[k], hipMemcpyHostToDevice);
            printf("%s{\"rep\": %d, \"bytes\": %zu, \"h2d_ms\": %.3f}", rep || k ? ", " : "", rep, sizes[k], ms_since(t0));
        }
    for (size_t k = 0; k < sizeof(sizes) / sizeof(sizes[0]); ++k) {
        auto t0 = std::chrono::steady_clock::now();
        (void)hipMemcpy(host, dev, sizes[k], hipMemcpyDeviceToHost);
        printf(", {\"bytes\": %zu, \"d2h_ms\": %.3f}", sizes[k], ms_since(t0));
    }
    printf("]\n");
    return 0;
}
