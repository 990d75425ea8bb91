/* Exhaustive check of nxc::div_by_n (libbicos_amd/csrc/nxc.hpp): RN(s/n) == fma-corrected
 * RN(s * RN(1/n)) for every integer s in [0, 65535 n], 2 <= n <= 65.
 *   gcc -O2 -ffp-contract=off tools/div_by_n_check.c -lm && ./a.out */
#include <stdio.h>
#include <math.h>
int main(void) {
    long bad = 0, tot = 0;
    for (int n = 2; n <= 65; ++n) {
        const float nf = (float)n;
        const float y = 1.0f / nf;  /* RN(1/n) */
        for (long s = 0; s <= 65535L * n; ++s) {
            const float sf = (float)s;
            const float ref = sf / nf;
            const float q0 = sf * y;
            const float r = fmaf(-q0, nf, sf);
            const float q = fmaf(r, y, q0);
            ++tot;
            if (q != ref) { if (bad < 5) printf("n=%d s=%ld ref=%a q=%a\n", n, s, ref, q); ++bad; }
        }
    }
    printf("checked %ld, bad %ld\n", tot, bad);
    return 0;
}
