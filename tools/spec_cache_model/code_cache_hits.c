#include <stdio.h>
#include <stdlib.h>
#include "../../gps-sdr-sim_amd/csrc/common/gss_phase.h"
/* code cycle-cache behaviour over whole blocks: hits on the previous cycle's entry, on its
   successor, on another entry, misses */
int main(void) {
    srand(1);
    long cyc = 0, same = 0, succ = 0, other = 0, miss = 0;
    for (int t = 0; t < 2000; t++) {
        double cs = 1.023e6 * (1.0 + ((rand() / (double)RAND_MAX) - 0.5) * 2e-5) / 2.6e6;
        double c0 = 1023.0 * (rand() / (double)RAND_MAX);
        gss_code_state st = {c0, 0, 0, 0};
        gss_code_it it; gss_code_it_init(&it, st, cs, 260000);
        int prev = -1, prevsucc = -1;
        /* first partial */
        gss_code_next_wrap(&it);
        while (it.left > 0) {
            int last_before = it.cc.last;
            int ps = last_before >= 0 ? it.cc.e[last_before].succ : -1;
            int n_before = it.cc.n;
            int next_before = it.cc.next;
            if (!gss_code_next_wrap(&it)) break;
            cyc++;
            int now = it.cc.last;
            if (it.cc.n != n_before || it.cc.next != next_before) miss++;
            else if (now == last_before) same++;
            else if (now == ps) succ++;
            else other++;
            (void)prev; (void)prevsucc;
        }
    }
    printf("cycles %ld: same entry %.3f, successor %.3f, other %.3f, miss %.3f\n", cyc, same/(double)cyc, succ/(double)cyc, other/(double)cyc, miss/(double)cyc);
    return 0;
}
