#include <rocrand/rocrand_philox4x32_10.h>
#include <cstdio>
int main(int argc, char** argv) {
    // stream spec: rocrand_init(seed, (sample<<32)|pixel, 0); first 12 draws
    unsigned long long seeds[3] = {1010ull, 0ull, 0x123456789abcdefull};
    unsigned pixels[3] = {0u, 1079999u, 77u};
    unsigned samples[3] = {0u, 999u, 5u};
    for (int t = 0; t < 3; ++t) {
        rocrand_state_philox4x32_10 st;
        rocrand_init(seeds[t], ((unsigned long long)samples[t] << 32) | pixels[t], 0, &st);
        printf("%llu %u %u", seeds[t], pixels[t], samples[t]);
        for (int i = 0; i < 12; ++i) printf(" %u", rocrand(&st));
        printf("\n");
    }
    return 0;
}
