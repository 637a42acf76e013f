// Probe: does a D2H copy issued straight to an SDMA engine (hsa_amd_memory_async_copy_on_engine)
// leave co-running kernels alone, where HIP's D2H (a __amd_rocclr_copyBuffer blit kernel) does not?
//   hipcc --offload-arch=gfx950 -O2 tools/sdma_probe.cpp -lhsa-runtime64 -o tools/sdma_probe
// Prints one line per case: copy ms, GB/s, and the per-launch ms of two victim kernels (an
// HBM-streaming copy and a latency-bound dependent-load kernel) run on a second stream.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <atomic>

#define HC(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
#define SC(x) do { hsa_status_t e = (x); if (e != HSA_STATUS_SUCCESS) { const char* s; hsa_status_string(e, &s); printf("HSA %s at %d\n", s, __LINE__); exit(1); } } while (0)

__global__ void stream_kernel(const float4* __restrict__ a, float4* __restrict__ b, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}
// latency-bound: each thread walks a chain of dependent loads
__global__ void chase_kernel(const int* __restrict__ nxt, int* __restrict__ out, int steps, int n) {
    int p = (blockIdx.x * blockDim.x + threadIdx.x) % n;
    for (int s = 0; s < steps; ++s) p = nxt[p];
    out[blockIdx.x * blockDim.x + threadIdx.x] = p;
}

static hsa_agent_t g_cpu;
static hsa_status_t find_cpu(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU) { g_cpu = a; return HSA_STATUS_INFO_BREAK; }
    return HSA_STATUS_SUCCESS;
}

int main() {
    const size_t bytes = 256ull << 20;
    float *src, *dst;
    HC(hipMalloc(&src, bytes));
    HC(hipHostMalloc(&dst, bytes, hipHostMallocDefault));
    HC(hipMemset(src, 1, bytes));
    const long nv = 64l << 20;   // 1 GiB / 16 B
    float4 *va, *vb;
    HC(hipMalloc(&va, nv * 16)); HC(hipMalloc(&vb, nv * 16));
    HC(hipMemset(va, 0, nv * 16));
    const int nchase = 1 << 22;
    int* nxt = (int*)malloc(nchase * 4);
    for (int i = 0; i < nchase; ++i) nxt[i] = (int)((i * 2654435761ull + 12345) % nchase);
    int *dn, *dout;
    HC(hipMalloc(&dn, nchase * 4)); HC(hipMalloc(&dout, 1 << 20));
    HC(hipMemcpy(dn, nxt, nchase * 4, hipMemcpyHostToDevice));

    hsa_amd_pointer_info_t info = {};
    info.size = sizeof(info);
    SC(hsa_amd_pointer_info(src, &info, nullptr, nullptr, nullptr));
    hsa_agent_t gpu = info.agentOwner;
    hsa_iterate_agents(find_cpu, nullptr);
    uint32_t mask = 0, rec = 0;
    hsa_status_t st = hsa_amd_memory_copy_engine_status(g_cpu, gpu, &mask);
    hsa_amd_memory_get_preferred_copy_engine(g_cpu, gpu, &rec);
    printf("engine_status %d mask 0x%x preferred 0x%x\n", (int)st, mask, rec);

    hipStream_t sc, sk;
    HC(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    HC(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0)); HC(hipEventCreate(&e1));

    auto victims = [&](int which, int reps) {   // ms per launch
        HC(hipEventRecord(e0, sk));
        for (int r = 0; r < reps; ++r) {
            if (which == 0) hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, sk, va, vb, nv);
            else hipLaunchKernelGGL(chase_kernel, dim3(512), dim3(256), 0, sk, dn, dout, 400, nchase);
        }
        HC(hipEventRecord(e1, sk));
        HC(hipEventSynchronize(e1));
        float ms; HC(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    hsa_signal_t sig;
    SC(hsa_signal_create(1, 0, nullptr, &sig));
    auto hsa_copy = [&](int engine) {
        hsa_signal_store_relaxed(sig, 1);
        if (engine < 0) SC(hsa_amd_memory_async_copy(dst, g_cpu, src, gpu, bytes, 0, nullptr, sig));
        else SC(hsa_amd_memory_async_copy_on_engine(dst, g_cpu, src, gpu, bytes, 0, nullptr, sig,
                                                   (hsa_amd_sdma_engine_id_t)engine, true));
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    };
    auto hip_copy = [&]() {
        HC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, sc));
        HC(hipStreamSynchronize(sc));
    };
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto msd = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    int eng = 0;
    for (int k = 0; k < 16; ++k) if ((rec ? rec : mask) & (1u << k)) { eng = 1 << k; break; }

    // warm
    hip_copy(); hsa_copy(-1); if (eng) hsa_copy(eng); victims(0, 2); victims(1, 2);
    for (int rep = 0; rep < 2; ++rep) {
        float v0 = victims(0, 20), v1 = victims(1, 20);
        printf("alone: stream %.3f ms  chase %.3f ms\n", v0, v1);
        for (int mode = 0; mode < 3; ++mode) {
            if (mode == 2 && !eng) continue;
            auto t0 = now();
            if (mode == 0) hip_copy(); else hsa_copy(mode == 1 ? -1 : eng);
            double cms = msd(t0, now());
            for (int w = 0; w < 2; ++w) {
                std::atomic<bool> stop{false};
                std::atomic<int> ncopies{0};
                std::thread th([&] { while (!stop) { if (mode == 0) hip_copy(); else hsa_copy(mode == 1 ? -1 : eng); ++ncopies; } });
                std::this_thread::sleep_for(std::chrono::milliseconds(20));
                float v = victims(w, 20);
                stop = true; th.join();
                printf("%-10s copy %.2f ms (%.1f GB/s alone)  victim %-6s %.3f ms per launch under copy (%d copies)\n",
                       mode == 0 ? "hip" : mode == 1 ? "hsa-auto" : "hsa-eng", cms, bytes / cms / 1e6,
                       w == 0 ? "stream" : "chase", v, (int)ncopies);
            }
        }
    }
    hsa_signal_destroy(sig);
    return 0;
}
