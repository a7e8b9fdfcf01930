// Probe of gfx950 buffer_load_dword ... lds (LDS-DMA) semantics used by k_tbn's A/B staging:
//  * destination = M0 + 4 * lane (lane-linear), also above 64 KiB of LDS
//  * out-of-range lanes (offset >= num_records): is 0 written or is LDS left untouched?
//  * exec-masked lanes: untouched
// Build: hipcc --offload-arch=gfx950 -O3 lds_dma_probe.hip -o lds_dma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kN = 40960;  // 160 KiB of floats
__global__ void probe(const float* g, float* out, unsigned nbytes, unsigned base_dw) {
    __shared__ float lds[kN];
    for (int q = threadIdx.x; q < kN; q += blockDim.x) lds[q] = -1.0f;
    __syncthreads();
    auto r = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, int(nbytes), 0x00020000);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (w == 0) {
        // A: lanes 0..31 in range, 32..63 out of range (offset 0x80000000)
        unsigned off = lane < 32 ? lane * 4u : 0x80000000u;
        unsigned m0 = (unsigned)(uintptr_t)(lds + base_dw);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, 0 offen lds" ::"v"(off), "s"(m0), "s"(r) : "memory");
        // B: exec-masked: lanes < 18 active, at base + 64
        if (lane < 18) {
            unsigned off2 = 256u + lane * 4u;
            unsigned m1 = (unsigned)(uintptr_t)(lds + base_dw + 64);
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, 0 offen lds" ::"v"(off2), "s"(m1), "s"(r) : "memory");
        }
        // C: whole wave out of range via num_records = 0 descriptor at base + 128
        auto r0 = __builtin_amdgcn_make_buffer_rsrc((void*)g, (short)0, 0, 0x00020000);
        unsigned m2 = (unsigned)(uintptr_t)(lds + base_dw + 128);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, 0 offen lds" ::"v"(lane * 4u), "s"(m2), "s"(r0) : "memory");
        // D: instruction offset 256 B: added to the source AND to the LDS address? at base + 192
        unsigned m3 = (unsigned)(uintptr_t)(lds + base_dw + 192);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, 0 offen offset:256 lds" ::"v"(lane * 4u), "s"(m3), "s"(r) : "memory");
        // E: dwordx4 pieces (16 B per lane) to an LDS address that is 8 mod 16, at base + 330
        //    (dwords): the 8-B-aligned destination an odd fp64 row pitch gives every other row
        unsigned m4 = (unsigned)(uintptr_t)(lds + base_dw + 330);
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds" ::"v"(lane * 16u), "s"(m4), "s"(r) : "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int q = threadIdx.x; q < 600; q += blockDim.x) out[q] = lds[base_dw + q];
}

int main() {
    float h[1024];
    for (int q = 0; q < 1024; ++q) h[q] = 1000.0f + q;
    float *g, *o;
    hipMalloc(&g, sizeof h);
    hipMalloc(&o, 600 * sizeof(float));
    hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
    int bad = 0;
    for (unsigned base : {0u, 16400u, 40000u}) {  // 0, ~64 KiB, ~156 KiB
        hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, g, o, unsigned(sizeof h), base);
        float r[600];
        hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
        int inr = 0, oobz = 0, oobu = 0, mk = 0, mu = 0, c0 = 0, cu = 0;
        for (int q = 0; q < 32; ++q) inr += r[q] == 1000.0f + q;
        for (int q = 32; q < 64; ++q) oobz += r[q] == 0.0f, oobu += r[q] == -1.0f;
        for (int q = 0; q < 18; ++q) mk += r[64 + q] == 1064.0f + q;
        for (int q = 18; q < 64; ++q) mu += r[64 + q] == -1.0f;
        for (int q = 0; q < 64; ++q) c0 += r[128 + q] == 0.0f, cu += r[128 + q] == -1.0f;
        int d_both = 0, d_src = 0;
        for (int q = 0; q < 64; ++q) d_both += r[192 + 64 + q] == 1064.0f + q, d_src += r[192 + q] == 1064.0f + q;
        int x4 = 0;
        for (int q = 0; q < 256; ++q) x4 += r[330 + q] == 1000.0f + q;
        printf("dwordx4 to an 8-mod-16 LDS address: %d/256 dwords where expected, guard before %s after %s\n", x4,
               r[329] == -1.0f ? "ok" : "CLOBBERED", r[586] == -1.0f ? "ok" : "CLOBBERED");
        bad += x4 != 256;
        printf("offset:256 -> LDS+256 & src+256: %d/64, LDS+0 & src+256: %d/64\n", d_both, d_src);
        printf("base_dw=%u in-range ok %d/32 | oob lanes: zero %d untouched %d | masked: active ok %d/18 untouched %d/46 | "
               "0-record desc: zero %d untouched %d\n", base, inr, oobz, oobu, mk, mu, c0, cu);
        bad += inr != 32 || mk != 18 || mu != 46;
    }
    printf(bad ? "PROBE FAIL\n" : "PROBE OK\n");
    return bad != 0;
}
