// lane-reduction check: v = 2^lane-ish distinct values; after row_ror:8 add and cross_rows, lane l
// should hold the sum over lanes {l ^ 8, 16, 32 combinations} (8 lanes with equal bits 0..2)
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../wavernn_amd/csrc/wrnn_device.h"
#include "../../wavernn_amd/csrc/xcd_device.h"
using namespace wrnn;
__global__ void k(float *out) {
    const int l = threadIdx.x;
    float v = (float)(l * l + 1);
    float a = v + WRNN_DPP(v, 0x128);
    out[l] = a;
    out[64 + l] = cross_rows(a);
}
int main() {
    float *d; hipMalloc(&d, 128 * 4);
    k<<<1, 64>>>(d);
    float h[128]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        float e1 = (float)(l * l + 1) + (float)((l ^ 8) * (l ^ 8) + 1);
        float e2 = 0; for (int m = 0; m < 64; ++m) if ((m & 7) == (l & 7)) e2 += (float)(m * m + 1);
        if (h[l] != e1 || h[64 + l] != e2) { if (bad < 8) printf("lane %d: ror %g (exp %g) all %g (exp %g)\n", l, h[l], e1, h[64+l], e2); ++bad; }
    }
    printf("bad lanes: %d\n", bad);
    return 0;
}
