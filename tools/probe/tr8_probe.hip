// Probe of ds_read_b64_tr_b8 / ds_read_b64_tr_b16 semantics on gfx950 (one wave): LDS byte i = i & 0xff
// (plus row tags), each lane supplies the address given by the mode, prints per-lane 8 received bytes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((ext_vector_type(2))) int i32x2;
typedef __attribute__((address_space(3))) i32x2 lds_i2;
__global__ void probe(uint8_t* out, int mode) {
    __shared__ __attribute__((aligned(16))) uint8_t s[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) s[i] = (uint8_t)((i / 128) * 16 + (i % 16));  // row r = i/128 (128-B rows), col c = i%128
    __syncthreads();
    const int lane = threadIdx.x;
    // mode 0: lane 2q+p within each 16-lane group -> row q (0..7) of the group's block, bytes 8p..8p+7;
    //         group g = lane/16 -> block rows 8g.. (guess for tr_b8)
    int q = (lane & 15) >> 1, p = lane & 1, g = lane >> 4;
    int addr = (8 * g + q) * 128 + 8 * p;
    if (mode == 1) addr = (lane & 15) * 128 + 8 * g;  // alternative: lane i -> row i
    i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i2*)(s + addr));
    uint8_t b[8];
    __builtin_memcpy(b, &v, 8);
    for (int k = 0; k < 8; ++k) out[lane * 8 + k] = b[k];
}
int main() {
    uint8_t* d; hipMalloc(&d, 512);
    uint8_t h[512];
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
        printf("mode %d (byte = 16*row + col%%16):\n", mode);
        for (int l = 0; l < 64; ++l) {
            printf("lane %2d:", l);
            for (int k = 0; k < 8; ++k) printf(" %02x", h[l * 8 + k]);
            printf("\n");
        }
    }
    return 0;
}
