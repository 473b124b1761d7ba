// Diagnostic (not shipped): cycles per step of dependent instruction chains typical of the rANS symbol
// loop, one wave, s_memtime (calibrated against s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k_chain(unsigned long long* out, const unsigned short* tab, int iters) {
    __shared__ unsigned short l[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) l[i] = tab[i];
    __syncthreads();
    const int lane = threadIdx.x;
    unsigned long long x = 0x123456789ull;
    unsigned v = lane * 7 + 3;
    unsigned s = __builtin_amdgcn_readfirstlane(iters) & 5;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if constexpr (MODE == 0) {          // SALU 64-bit mul-add on a uniform state
                unsigned f = (unsigned)(x & 0xfff) + 1;
                x = (unsigned long long)f * (x >> 16) + (x & 0xffff);
                x = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(x >> 32)) << 32) | __builtin_amdgcn_readfirstlane((unsigned)x);
            } else if constexpr (MODE == 1) {   // v_readlane with SGPR lane select feeding the next select
                s = __builtin_amdgcn_readlane(v, s & 63);
            } else if constexpr (MODE == 2) {   // uniform LDS read -> readfirstlane -> next address
                s = __builtin_amdgcn_readfirstlane(l[(s & 4095)]);
            } else if constexpr (MODE == 3) {   // window LDS read + compare + ballot + popcount
                const unsigned c = l[(s + lane) & 4095];
                s = (unsigned)__popcll(__ballot(c <= (s & 0xffff))) + s;
            } else if constexpr (MODE == 4) {   // 64-bit compare + data-dependent branch + renorm
                if (x < (1ull << 31)) x = (x << 32) | s; else x = x - 12345;
                x = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(x >> 32)) << 32) | __builtin_amdgcn_readfirstlane((unsigned)x);
            } else if constexpr (MODE == 5) {   // dependent s_add
                asm volatile("s_add_u32 %0, %0, 1" : "+s"(s));
            } else if constexpr (MODE == 6) {   // dependent v_add
                asm volatile("v_add_u32 %0, %0, 1" : "+v"(v));
            } else if constexpr (MODE == 7) {   // v_add -> readfirstlane -> s_add (VALU->SALU round trip)
                v += s;
                s = __builtin_amdgcn_readfirstlane(v) + 1;
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) { out[0] = t1 - t0; out[1] = x + s + v; out[2] = r1 - r0; }
}

template <int MODE>
void run(const char* name, unsigned long long* out, unsigned short* tab) {
    unsigned long long h[3];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_chain<MODE>, dim3(1), dim3(64), 0, nullptr, out, tab, 2000);
        (void)hipMemcpy(h, out, 24, hipMemcpyDeviceToHost);
    }
    printf("%-44s %6.1f cycles/step (%.2f GHz)\n", name, h[0] / 16000.0, h[0] / (h[2] * 10.0));
}

int main() {
    unsigned long long* out;
    unsigned short* tab;
    (void)hipMalloc(&out, 32);
    (void)hipMalloc(&tab, 8192);
    (void)hipMemset(tab, 1, 8192);
    run<0>("salu 64b mul-add + readfirstlane x2", out, tab);
    run<1>("v_readlane sgpr-select", out, tab);
    run<2>("uniform lds read + readfirstlane", out, tab);
    run<3>("window lds read + cmp + ballot + popc", out, tab);
    run<4>("64b compare + branch + renorm", out, tab);
    run<5>("dependent s_add", out, tab);
    run<6>("dependent v_add", out, tab);
    run<7>("v_add -> readfirstlane -> s_add", out, tab);
    return 0;
}
