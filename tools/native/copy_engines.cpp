// Diagnostic: which engine moves a host<->device copy.  hipMemcpyAsync with
// page-locked host memory (hipHostMalloc) against hsa_amd_memory_async_copy
// (a DMA engine, no shader), timed per direction; run it under
// rocprofv3 --kernel-trace to see which of them launch __amd_rocclr_copyBuffer
// kernels on the CUs.
//   hipcc --offload-arch=gfx950 -O2 -o copy_engines copy_engines.cpp -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
    const size_t chunk = (size_t)(argc > 1 ? atoi(argv[1]) : 32) << 20;
    const int reps = 16;
    for (const char *v : {"HSA_ENABLE_SDMA", "ROC_ENABLE_LARGE_BAR", "GPU_FORCE_BLIT_COPY_SIZE", "HIP_FORCE_DEV_KERNARG"}) {
        const char *e = getenv(v);
        printf("env %s=%s\n", v, e ? e : "(unset)");
    }
    hipSetDevice(0);
    uint8_t *h = nullptr, *d = nullptr;
    hipHostMalloc((void **)&h, chunk * 2, hipHostMallocDefault);
    hipMalloc((void **)&d, chunk * 2);
    for (size_t i = 0; i < chunk * 2; ++i) h[i] = (uint8_t)i;
    int lo_pri = 0, hi_pri = 0;
    hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri);
    printf("stream priorities: least %d greatest %d\n", lo_pri, hi_pri);
    for (int pri = 0; pri < 2; ++pri) {
    hipStream_t s;
    if (pri) hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi_pri);
    else hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int dir = 0; dir < 2; ++dir) {
        hipStreamSynchronize(s);
        double t0 = now();
        for (int r = 0; r < reps; ++r) {
            if (dir == 0) hipMemcpyAsync(d + (r & 1) * chunk, h + (r & 1) * chunk, chunk, hipMemcpyHostToDevice, s);
            else hipMemcpyAsync(h + (r & 1) * chunk, d + (r & 1) * chunk, chunk, hipMemcpyDeviceToHost, s);
        }
        hipStreamSynchronize(s);
        double dt = now() - t0;
        printf("hipMemcpyAsync %s%s: %.1f GB/s (%d x %zu MiB)\n", dir ? "D2H" : "H2D", pri ? " (highest-priority stream)" : "",
               reps * chunk / dt / 1e9, reps, chunk >> 20);
    }
    hipStreamDestroy(s);
    }
    if (hsa_iterate_agents(find_agents, nullptr) != HSA_STATUS_SUCCESS || !g_gpu.handle || !g_cpu.handle) {
        printf("hsa agents not found\n");
        return 1;
    }
    hsa_signal_t sig;
    hsa_signal_create(1, 0, nullptr, &sig);
    for (int dir = 0; dir < 2; ++dir) {
        double t0 = now();
        for (int r = 0; r < reps; ++r) {
            hsa_signal_store_relaxed(sig, 1);
            hsa_status_t st;
            if (dir == 0) st = hsa_amd_memory_async_copy(d + (r & 1) * chunk, g_gpu, h + (r & 1) * chunk, g_cpu, chunk, 0, nullptr, sig);
            else st = hsa_amd_memory_async_copy(h + (r & 1) * chunk, g_cpu, d + (r & 1) * chunk, g_gpu, chunk, 0, nullptr, sig);
            if (st != HSA_STATUS_SUCCESS) { printf("hsa copy failed %d\n", (int)st); return 1; }
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        }
        double dt = now() - t0;
        printf("hsa_amd_memory_async_copy %s: %.1f GB/s\n", dir ? "D2H" : "H2D", reps * chunk / dt / 1e9);
    }
    // check the last D2H landed
    bool ok = true;
    for (size_t i = 0; i < chunk; i += 4097) ok &= h[i] == (uint8_t)i;
    printf("data %s\n", ok ? "ok" : "MISMATCH");
    hsa_signal_destroy(sig);
    hipFree(d);
    hipHostFree(h);
    return 0;
}
