/* oracle_sanitize.c -- the CPU checker (oracle/turbo_oracle.c) under AddressSanitizer and
 * UndefinedBehaviorSanitizer (built by tests/test_host_sanitizers.py).  Decodes a
 * seeded batch at K = 40 and K = 1024 in both algorithms and precisions, threaded, plus the
 * SISO and the channel, and prints a checksum of the decisions that the test compares with the
 * uninstrumented liboracle.so on the same inputs. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "turbo_oracle.h"

int main(void)
{
    unsigned long long sum = 0;
    const int Ks[2] = {40, 1024}, f1s[2] = {3, 31}, f2s[2] = {10, 64};
    for (int k = 0; k < 2; ++k) {
        const int K = Ks[k], B = 5, n = 3 * K + 12;
        int* src = malloc(sizeof(int) * (size_t)B * K);
        double* flow = malloc(sizeof(double) * (size_t)B * n);
        float* flow32 = malloc(sizeof(float) * (size_t)B * n);
        uint8_t* bits = malloc((size_t)B * K);
        tdo_synth_batch(K, f1s[k], f2s[k], 0.4, 77 + k, B, src, flow);
        for (int i = 0; i < B * n; ++i) flow32[i] = (float)flow[i];
        for (int algo = 0; algo < 2; ++algo)
            for (int f32 = 0; f32 < 2; ++f32) {
                tdo_decode_batch(K, f1s[k], f2s[k], 3, algo, f32, f32 ? (const void*)flow32 : (const void*)flow, B, bits, 2);
                for (int i = 0; i < B * K; ++i) sum = sum * 1000003ull + bits[i];
            }
        free(src);
        free(flow);
        free(flow32);
        free(bits);
    }
    printf("%llu\n", sum);
    return 0;
}
