// Phase timing of the fused per-agent MLP kernel (csrc/mlp_fused.hip): runs it on c3's shapes
// (256 agents, B 64, 784-150-10) with per-workgroup wall-clock stamps and prints the mean
// duration of each phase.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//   -I distributed-learning_amd/csrc -o scripts/mlp_probe scripts/mlp_probe.hip
//   distributed-learning_amd/_lib/obj/capi.o ... (see scripts/gpu_mlp_probe.sh)
#include <cstdio>
#include <vector>

#include "../distributed-learning_amd/csrc/mlp_fused.hip"

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

namespace dl {
hipError_t allow_full_lds(const void *k) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
}
}  // namespace dl

int main(int argc, char **argv) {
    // argv[1] == "fp32": layer 1 and dW1 on the fp32 MFMA (default: the bf16x6 split)
    const bool x6 = !(argc > 1 && argv[1][0] == 'f');
    // argv[2] == "tiled": X and G in the engine's column-tiled layout (T = 64 for 256 agents)
    const bool tiled = argc > 2 && argv[2][0] == 't';
    // argv[3] == "step": G receives the local step x - lr g (dl_mlp_args.out_mode 1)
    const bool step = argc > 3 && argv[3][0] == 's';
    auto kern = step ? (tiled ? (x6 ? dl::mlp_fused_kernel<true, true, true>
                                    : dl::mlp_fused_kernel<true, false, true>)
                              : (x6 ? dl::mlp_fused_kernel<false, true, true>
                                    : dl::mlp_fused_kernel<false, false, true>))
                     : (tiled ? (x6 ? dl::mlp_fused_kernel<true, true, false>
                                    : dl::mlp_fused_kernel<true, false, false>)
                              : (x6 ? dl::mlp_fused_kernel<false, true, false>
                                    : dl::mlp_fused_kernel<false, false, false>));
    const int N = 256, B = 64, din = 784, dh = 150, dout = 10;
    const long P = (long)dh * din + dh + 2 * (dh * dh + dh) + dout * dh + dout;
    const long ld = (P + 63) / 64 * 64;
    std::vector<float> hx(N * ld), hd((long)N * B * din);
    std::vector<int> hl(N * B);
    unsigned s = 1;
    auto rnd = [&] { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.f - 0.5f; };
    for (auto &v : hx) v = 0.1f * rnd();
    for (auto &v : hd) v = rnd();
    for (auto &v : hl) v = (int)((rnd() + 0.5f) * dout) % dout;
    float *X, *D, *G, *L;
    int *Y;
    uint64_t *st;
    CHECK(hipMalloc(&X, hx.size() * 4));
    CHECK(hipMalloc(&D, hd.size() * 4));
    CHECK(hipMalloc(&G, hx.size() * 4));
    CHECK(hipMalloc(&L, N * 4));
    CHECK(hipMalloc(&Y, N * B * 4));
    CHECK(hipMalloc(&st, N * 16 * 8));
    CHECK(hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(D, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(Y, hl.data(), hl.size() * 4, hipMemcpyHostToDevice));
    CHECK(dl::allow_full_lds(reinterpret_cast<const void *>(kern)));
    // tiled: T = 64 -> tsh 6, tile stride N * 64 floats (ld is a multiple of 64: whole tiles)
    dl::MlpArgs p{X, ld, D, (long)B * din, Y, B, G, ld, L, din, dh, dout, tiled ? 6 : 0,
                  tiled ? (long)N * 64 : 0, st, 0.05f};
    int rate_khz = 0;
    CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const char *names[] = {"layer1 fwd", "fwd2", "fwd3", "logits+xent", "dW4+db4+dZ3", "dW3",
                           "dZ2", "dW2", "dZ1", "dW1"};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 6; ++rep) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(N), dim3(dl::NTHR),
                           dl::LDS_FLOATS * sizeof(float), 0, p);
        CHECK(hipEventRecord(e1));
        CHECK(hipDeviceSynchronize());
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<uint64_t> hs(N * 16);
        CHECK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
        double ph[10] = {0}, tot = 0, clk = 0;
        uint64_t t0min = ~0ull, t1max = 0;
        for (int a = 0; a < N; ++a) {
            const uint64_t *t = &hs[a * 16];
            static const int idx[11] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
            for (int i = 0; i < 10; ++i) ph[i] += (double)(t[idx[i + 1]] - t[idx[i]]);
            tot += (double)(t[10] - t[0]);
            clk += (double)(t[15] - t[14]) / (double)(t[10] - t[0]) * rate_khz / 1e3;  // MHz
            t0min = t[0] < t0min ? t[0] : t0min;
            t1max = t[10] > t1max ? t[10] : t1max;
        }
        const double us = 1e3 / rate_khz;   // ticks -> us
        printf("rep %d: event %.1f us, wg span %.1f us, mean wg %.1f us, s_memtime %.0f MHz:",
               rep, ms * 1e3, (t1max - t0min) * us, tot / N * us, clk / N);
        for (int i = 0; i < 10; ++i) printf(" %s %.1f", names[i], ph[i] / N * us);
        printf("\n");
    }
    return 0;
}
