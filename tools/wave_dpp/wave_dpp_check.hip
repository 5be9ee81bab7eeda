// Checks kt::shfl_xor_{d,u64,i} (kt_wave.h) against __shfl_xor(v, o, 64) for
// o = 1 .. 32 on random bit patterns, and a full xor-butterfly sum of each
// form bit for bit.  Build: make -C tools/wave_dpp; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../../krylov_robustness_amd/csrc/kt_wave.h"

__global__ void k_check(const unsigned long long* in, int* bad) {
    const int l = threadIdx.x;
    const unsigned long long b = in[blockIdx.x * 64 + l];
    const double v = __longlong_as_double((long long)(b & 0x7FEFFFFFFFFFFFFFull));  // finite
    int nb = 0;
    for (int o = 1; o < 64; o <<= 1) {
        if (kt::shfl_xor_u64(b, o) != (unsigned long long)__shfl_xor(b, o, 64)) nb |= 1;
        if (kt::shfl_xor_i((int)b, o) != __shfl_xor((int)b, o, 64)) nb |= 2;
        const double x = kt::shfl_xor_d(v, o), y = __shfl_xor(v, o, 64);
        if (__double_as_longlong(x) != __double_as_longlong(y)) nb |= 4;
    }
    double s1 = v, s2 = v;
    for (int o = 32; o > 0; o >>= 1) {
        s1 += kt::shfl_xor_d(s1, o);
        s2 += __shfl_xor(s2, o, 64);
    }
    if (__double_as_longlong(s1) != __double_as_longlong(s2)) nb |= 8;
    if (nb) atomicOr(bad, nb);
}

int main() {
    const int blocks = 4096;
    unsigned long long* h = (unsigned long long*)malloc(sizeof(unsigned long long) * 64 * blocks);
    unsigned long long x = 88172645463325252ull;
    for (int i = 0; i < 64 * blocks; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        h[i] = x;
    }
    unsigned long long* d;
    int *db, hb = 0;
    if (hipMalloc(&d, sizeof(unsigned long long) * 64 * blocks) != hipSuccess || hipMalloc(&db, sizeof(int)) != hipSuccess)
        return 2;
    (void)hipMemcpy(d, h, sizeof(unsigned long long) * 64 * blocks, hipMemcpyHostToDevice);
    (void)hipMemset(db, 0, sizeof(int));
    k_check<<<blocks, 64>>>(d, db);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(&hb, db, sizeof(int), hipMemcpyDeviceToHost);
    printf("{\"wave_dpp_check\": \"%s\", \"mismatch_mask\": %d, \"lanes\": %d}\n", hb ? "FAIL" : "ok", hb, 64 * blocks);
    return hb ? 1 : 0;
}
