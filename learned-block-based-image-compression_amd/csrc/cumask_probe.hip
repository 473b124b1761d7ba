// Diagnostic (not part of liblbic.so): where the workgroups of a launch on a CU-masked stream run.
//   build: make cumask_probe      run: ./build/cumask_probe
// Each workgroup records its XCC_ID and HW_ID (CU / SH / SE), waits ~20 us (bounded) so the grid spreads, and the host
// prints, per mask, the CUs seen on every XCD; then the two complementary masks run at once.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void k_probe(unsigned* out) {
    if (threadIdx.x == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(10);   // 100 MHz: 20 us
        out[blockIdx.x * 2] = hw;
        out[blockIdx.x * 2 + 1] = xcc;
    }
}

static void report(const char* name, const std::vector<unsigned>& h, int n) {
    std::set<unsigned> cus[8];
    int cnt[8] = {0};
    for (int b = 0; b < n; ++b) {
        const unsigned hw = h[2 * b], x = h[2 * b + 1] & 7;
        const unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        cus[x].insert(se * 32 + sh * 16 + cu);
        ++cnt[x];
    }
    printf("%s:\n", name);
    for (int x = 0; x < 8; ++x) {
        printf("  xcc %d: %4d wgs on %2zu CUs:", x, cnt[x], cus[x].size());
        for (unsigned c : cus[x]) printf(" %u.%u.%u", c / 32, (c / 16) & 1, c & 15);
        printf("\n");
    }
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", cus);
    const int words = (cus + 31) / 32, n = 2048;
    std::vector<uint32_t> ma(words, 0), mb(words, 0);
    for (int i = 0; i < cus; ++i) ((i / 8) % 2 == 0 ? ma : mb)[i / 32] |= 1u << (i % 32);
    hipStream_t sa, sb;
    if (hipExtStreamCreateWithCUMask(&sa, words, ma.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&sb, words, mb.data()) != hipSuccess) {
        printf("hipExtStreamCreateWithCUMask failed\n");
        return 1;
    }
    unsigned *da, *db;
    (void)hipMalloc(&da, n * 2 * sizeof(unsigned));
    (void)hipMalloc(&db, n * 2 * sizeof(unsigned));
    std::vector<unsigned> ha(n * 2), hb(n * 2);
    hipLaunchKernelGGL(k_probe, dim3(n), dim3(64), 0, sa, da);
    (void)hipStreamSynchronize(sa);
    (void)hipMemcpy(ha.data(), da, n * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    report("mask A (bits i with (i/8)%2==0), alone", ha, n);
    hipLaunchKernelGGL(k_probe, dim3(n), dim3(64), 0, sb, db);
    (void)hipStreamSynchronize(sb);
    (void)hipMemcpy(hb.data(), db, n * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    report("mask B (complement), alone", hb, n);
    hipLaunchKernelGGL(k_probe, dim3(n), dim3(64), 0, sa, da);
    hipLaunchKernelGGL(k_probe, dim3(n), dim3(64), 0, sb, db);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(ha.data(), da, n * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hb.data(), db, n * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    report("mask A beside B", ha, n);
    report("mask B beside A", hb, n);
    hipStream_t s0;
    (void)hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
    hipLaunchKernelGGL(k_probe, dim3(n), dim3(64), 0, s0, da);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(ha.data(), da, n * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    report("unmasked", ha, n);
    return 0;
}
