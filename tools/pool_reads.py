"""Which stored pool arrays are ever read (diagnostic, CPU only).

Builds an instrumented copy of the oracle's loop-faithful SCL (oracle/refcpu.c)
that emulates the tree kernel's pointer rows: at leaf i every active path reads
its depth-(dstart-1) array (the g of the right child) and stores new arrays at
depths dstart..n-1; survivors inherit their parent's rows.  Prints, per
workspace depth 3..6, how many arrays were stored and how many distinct ones
were ever read -- the share of the pool store traffic that no later g reads.

usage: python tools/pool_reads.py [N L frames snr]
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HOOK_LEAF = "        if (frozen_mask[l]) {"
HOOK_PRUNE = "            for (int k = 0; k < ns; k++) {\n                const int op = cand[k].p;"
DECL = "long g_owner[1024][16]; char* g_read; long g_next; long g_nstore[16], g_nread[16];\n"
LEAF = """        {
            const int dst = (i == 0) ? 1 : n - __builtin_ctz(i);
            for (int p = 0; p < Lsz; p++) {
                if (!act[p]) continue;
                if (dst - 1 >= 3 && dst - 1 <= 6) { long id = g_owner[p][dst - 1]; if (!g_read[id]) { g_read[id] = 1; g_nread[dst - 1]++; } }
                for (int d = dst; d < n; d++) { g_owner[p][d] = g_next; g_read[g_next] = 0; g_next++; if (d >= 3 && d <= 6) g_nstore[d]++; }
            }
        }
"""
PRUNE = """            { static long tmp[1024][16]; for (int k = 0; k < ns; k++) memcpy(tmp[k], g_owner[cand[k].p], sizeof(tmp[k]));
              for (int k = 0; k < ns; k++) memcpy(g_owner[k], tmp[k], sizeof(tmp[k])); }
"""
MAIN = r"""
#include <stdio.h>
int main(int argc, char** argv) {
    int N = atoi(argv[1]), L = atoi(argv[2]), B = atoi(argv[3]);
    FILE* f = fopen(argv[4], "rb"); uint8_t* fr = malloc(N);
    double* llr = malloc(sizeof(double) * N * (size_t)B);
    if (fread(fr, 1, N, f) != (size_t)N || fread(llr, 8, (size_t)N * B, f) != (size_t)N * B) return 1;
    fclose(f);
    uint8_t* u = malloc(N);
    g_read = calloc(400000000, 1);
    for (int b = 0; b < B; b++) orc_scl_decode(N, L, fr, llr + (size_t)b * N, u);
    for (int d = 3; d <= 6; d++)
        printf("depth %d: arrays stored %ld, distinct arrays read %ld (%.3f)\n", d, g_nstore[d], g_nread[d],
               (double)g_nread[d] / g_nstore[d]);
    return 0;
}
"""


def main():
    N, L, B, snr = 1024, 8, 100, 3.0
    if len(sys.argv) > 4:
        N, L, B, snr = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
    src = open(os.path.join(ROOT, "oracle", "refcpu.c")).read()
    assert HOOK_LEAF in src and HOOK_PRUNE in src
    src = src.replace(HOOK_LEAF, LEAF + HOOK_LEAF).replace(HOOK_PRUNE, PRUNE + HOOK_PRUNE)
    src = src.replace("static int scl_decode_impl(", DECL + "static int scl_decode_impl(", 1) + MAIN
    from polarcode_and_ldpc_amd.polar import construct_frozen_set
    K = N // 2
    fr = np.zeros(N, np.uint8)
    fr[np.asarray(construct_frozen_set(N, K, 2.0))] = 1
    rs = np.random.RandomState(1)
    sig = np.sqrt(1 / (2 * 10 ** (snr / 10)))
    llr = 2 * (1 + sig * rs.randn(B, N)) / sig ** 2  # all-zero codeword (linear code, symmetric channel)
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "p.c"), "w").write(src)
        with open(os.path.join(d, "llr.bin"), "wb") as f:
            f.write(fr.tobytes())
            f.write(llr.astype(np.float64).tobytes())
        subprocess.check_call(["gcc", "-O2", "-I", os.path.join(ROOT, "oracle"), "-o", os.path.join(d, "p"),
                               os.path.join(d, "p.c"), "-lm"])
        print("N=%d L=%d frames=%d Es/N0=%.1f dB" % (N, L, B, snr), flush=True)
        subprocess.check_call([os.path.join(d, "p"), str(N), str(L), str(B), os.path.join(d, "llr.bin")])


if __name__ == "__main__":
    main()
