// Which XCD / CU the workgroups of a CU-masked stream land on (hipExtStreamCreateWithCUMask):
// each workgroup reads XCC_ID and HW_ID (vector stores only) and spins briefly so that
// the workgroups of one launch are resident together.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <set>

__global__ void probe(unsigned* out, unsigned long long spin) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < spin) {}
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = xcc; out[2 * blockIdx.x + 1] = hw; }
}

static void run(const char* name, const std::vector<uint32_t>& mask, int blocks) {
    hipStream_t s;
    if (mask.empty()) hipStreamCreate(&s);
    else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size() * 32, mask.data()) != hipSuccess) { printf("%s: mask failed\n", name); return; }
    unsigned* d; hipMalloc(&d, blocks * 8);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, s, d, 20000ull);
    hipStreamSynchronize(s);
    std::vector<unsigned> h(blocks * 2);
    hipMemcpy(h.data(), d, blocks * 8, hipMemcpyDeviceToHost);
    int per[8] = {0};
    std::set<unsigned> cus;
    for (int b = 0; b < blocks; ++b) { per[h[2*b] & 7]++; cus.insert(((h[2*b] & 7) << 16) | ((h[2*b+1] >> 8) & 0xF) | (((h[2*b+1] >> 13) & 7) << 4) | (((h[2*b+1] >> 12) & 1) << 7)); }
    printf("%s: blocks per xcc", name);
    for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
    printf(" | distinct (xcc,se,sh,cu) %zu | first blocks xcc:", cus.size());
    for (int b = 0; b < 16 && b < blocks; ++b) printf(" %u", h[2*b] & 7);
    printf("\n");
    hipFree(d); hipStreamDestroy(s);
}

int main() {
    int n_cu = 0; hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", n_cu);
    const int words = (n_cu + 31) / 32;
    run("nomask", {}, 256);
    std::vector<uint32_t> lo16(words, 0); lo16[0] = 0xFFFFu;  // bits 0..15
    run("bits0-15", lo16, 64);
    std::vector<uint32_t> rest(words, 0xFFFFFFFFu); rest[0] = 0xFFFF0000u;  // bits 16..
    run("bits16-", rest, 240);
    std::vector<uint32_t> b0(words, 0); b0[0] = 0xFFu;  // bits 0..7
    run("bits0-7", b0, 32);
    std::vector<uint32_t> b32(words, 0); b32[1] = 0xFFFFFFFFu;  // bits 32..63
    run("bits32-63", b32, 64);
    return 0;
}
