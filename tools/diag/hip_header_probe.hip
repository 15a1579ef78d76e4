// Which AQL header does HIP give a kernel?  Each kernel reads the first word of its own dispatch packet (header +
// setup, through the dispatch pointer) and stores it; launched three times back to back on a stream, then as three
// nodes of a captured hipGraph.  Header bits: 0-7 type (2 = kernel dispatch), 8 barrier, 9-10 acquire scope,
// 11-12 release scope (0 none, 1 agent, 2 system).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/diag/hip_header_probe tools/diag/hip_header_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_hdr(unsigned *out, int slot) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const __attribute__((address_space(4))) unsigned *pkt =
            (const __attribute__((address_space(4))) unsigned *)__builtin_amdgcn_dispatch_ptr();
        out[slot] = pkt[0];
    }
}

static void show(const char *what, const unsigned *h, int n) {
    for (int i = 0; i < n; ++i) {
        const unsigned w = h[i];
        std::printf("%-14s #%d  word 0x%08x  type %u barrier %u acquire %u release %u\n", what, i, w, w & 0xff,
                    (w >> 8) & 1, (w >> 9) & 3, (w >> 11) & 3);
    }
}

int main() {
    unsigned *d = nullptr, h[8] = {0};
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    (void)hipMemset(d, 0, 64);
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_hdr, dim3(2048), dim3(64), 0, st, d, i);
    (void)hipStreamSynchronize(st);
    (void)hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
    show("stream", h, 3);
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_hdr, dim3(2048), dim3(64), 0, st, d, 3 + i);
    (void)hipStreamEndCapture(st, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int r = 0; r < 2; ++r) (void)hipGraphLaunch(ge, st);
    (void)hipStreamSynchronize(st);
    (void)hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
    show("graph", h + 3, 3);
    return 0;
}
