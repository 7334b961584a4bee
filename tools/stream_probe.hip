// stream_probe.hip -- runtime facts the work-queue slot lifecycle rests on
// (mchecksum_gpu.hip, queue_slot), measured on the box:
//  1. does hipStreamGetId give a destroyed stream's successor a new id, when
//     hipStreamDestroy + hipStreamCreate hands back the same handle?
//  2. device + host cost of completion evidence per launch, on a series of
//     ~40 us streaming-read kernels (C2's size): plain launch; hipExtLaunchKernel
//     with a stop event; launch + hipEventRecord; hipStreamWaitEvent on the
//     stream's own previous event + launch.
// Build: hipcc -O2 --offload-arch=gfx950 tools/stream_probe.hip -o build/stream_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__global__ __launch_bounds__(256) void read_kernel(const uint4 *p, uint64_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads alive
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    // ---- 1. ids vs handles over create/destroy cycles
    int handle_reuse = 0, id_reuse = 0;
    std::set<unsigned long long> ids;
    hipStream_t prev = nullptr;
    for (int i = 0; i < 200; i++) {
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        unsigned long long id = 0;
        CK(hipStreamGetId(s, &id));
        if (s == prev) handle_reuse++;
        if (!ids.insert(id).second) id_reuse++;
        prev = s;
        CK(hipStreamDestroy(s));
    }
    unsigned long long id_null = 0, id_pt = 0;
    hipError_t e_null = hipStreamGetId(nullptr, &id_null);
    hipError_t e_pt = hipStreamGetId(hipStreamPerThread, &id_pt);
    printf("{\"cycles\": 200, \"handle_reused\": %d, \"id_reused\": %d, \"null_stream_id\": [%d, %llu], "
           "\"per_thread_id\": [%d, %llu]}\n",
           handle_reuse, id_reuse, (int)e_null, id_null, (int)e_pt, id_pt);
    // handle reuse while the old one has work in flight
    {
        const uint64_t n = (256ull << 20) / 16;
        uint4 *buf;
        uint32_t *sink;
        CK(hipMalloc(&buf, n * 16));
        CK(hipMemset(buf, 1, n * 16));
        CK(hipMalloc(&sink, 4));
        int reuse = 0, idsame = 0;
        for (int t = 0; t < 20; t++) {
            hipStream_t a, b;
            unsigned long long ia, ib;
            CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
            CK(hipStreamGetId(a, &ia));
            for (int k = 0; k < 10; k++) hipLaunchKernelGGL(read_kernel, dim3(2048), dim3(256), 0, a, buf, n, sink);
            CK(hipStreamDestroy(a));
            CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
            CK(hipStreamGetId(b, &ib));
            reuse += a == b;
            idsame += ia == ib;
            CK(hipStreamDestroy(b));
        }
        CK(hipDeviceSynchronize());
        printf("{\"in_flight_cycles\": 20, \"handle_reused\": %d, \"id_same\": %d}\n", reuse, idsame);
        CK(hipFree(buf));
        CK(hipFree(sink));
    }

    // ---- 2. completion-evidence cost per launch
    const uint64_t n = (256ull << 20) / 16;  // 256 MiB: ~40 us per launch
    uint4 *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, n * 16));
    CK(hipMemset(buf, 1, n * 16));
    CK(hipMalloc(&sink, 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t t0, t1, ev;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const unsigned grid = 2048;
    void *args[] = {&buf, (void *)&n, &sink};
    const char *names[] = {"plain", "ext_stop_event", "launch_then_record", "wait_own_event_then_launch", "plain_again"};
    const int L = 200;
    for (int rep = 0; rep < 3; rep++) {
        for (int mode = 0; mode < 5; mode++) {
            for (int w = 0; w < 40; w++) hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, s, buf, n, sink);
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(t0, s));
            const double h0 = now_us();
            for (int i = 0; i < L; i++) {
                switch (mode) {
                    case 1:
                        CK(hipExtLaunchKernel((const void *)read_kernel, dim3(grid), dim3(256), args, 0, s, nullptr, ev, 0));
                        break;
                    case 2:
                        hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, s, buf, n, sink);
                        CK(hipEventRecord(ev, s));
                        break;
                    case 3:
                        if (i) CK(hipStreamWaitEvent(s, ev, 0));
                        hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, s, buf, n, sink);
                        CK(hipEventRecord(ev, s));
                        break;
                    default:
                        hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, s, buf, n, sink);
                }
            }
            const double h1 = now_us();
            CK(hipEventRecord(t1, s));
            CK(hipStreamSynchronize(s));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            hipError_t q = hipEventQuery(ev);
            printf("{\"rep\": %d, \"mode\": \"%s\", \"device_us_per_launch\": %.3f, \"host_us_per_call\": %.3f, "
                   "\"ev_query_after_sync\": %d}\n",
                   rep, names[mode], ms * 1e3 / L, (h1 - h0) / L, (int)q);
        }
    }
    // hipEventQuery cost (complete event)
    const double q0 = now_us();
    for (int i = 0; i < 10000; i++) (void)hipEventQuery(ev);
    printf("{\"event_query_us\": %.4f}\n", (now_us() - q0) / 10000);
    const double g0 = now_us();
    unsigned long long id;
    for (int i = 0; i < 10000; i++) (void)hipStreamGetId(s, &id);
    printf("{\"stream_get_id_us\": %.4f}\n", (now_us() - g0) / 10000);
    return 0;
}
