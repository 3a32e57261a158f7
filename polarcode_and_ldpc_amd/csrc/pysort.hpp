// CPython 3.10 list.sort(key=..., reverse=True) as a single-thread device
// routine over an LDS array, for SCL candidate lists with NaN path metrics
// (polar_nan.hip).  The reference sorts its candidates with that call
// (src/polar/decoder.py:306-307); for finite keys the result is the stable
// descending order the fast kernels compute in parallel, but a NaN key compares
// false both ways and the order CPython leaves depends on its exact algorithm:
// reverse, count_run + binary insertion below minrun, runs merged by
// merge_collapse with merge_lo / merge_hi and galloping (MIN_GALLOP 7),
// reverse (Objects/listobject.c).  Every step here compares with `<` only, in
// CPython's order.  Checked against the interpreter through the oracle's
// restatement (tests/test_oracle_golden.py::test_pysort_matches_cpython) and on
// reference decodes of NaN frames (tests/test_gpu_polar.py::test_scl_nan_metrics_golden).
#pragma once
#include "common.hpp"

namespace pl {

struct PsItem {
    double k;
    int v;
    int pad;
};

namespace pysort {

constexpr int kMinGallop = 7;
constexpr int kMaxPending = 40;  // runs pending on the stack: ample for n <= 2^15

PL_DEV bool lt(const PsItem& a, const PsItem& b) { return a.k < b.k; }

PL_DEV void copy_fwd(PsItem* d, const PsItem* s, int n) {
    for (int i = 0; i < n; ++i) d[i] = s[i];
}
PL_DEV void copy_bwd(PsItem* d, const PsItem* s, int n) {
    for (int i = n - 1; i >= 0; --i) d[i] = s[i];
}
PL_DEV void reverse(PsItem* a, int n) {
    for (int i = 0, j = n - 1; i < j; ++i, --j) {
        const PsItem t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
}

PL_DEV int minrun(int n) {
    int r = 0;
    while (n >= 64) {
        r |= n & 1;
        n >>= 1;
    }
    return n + r;
}

PL_DEV int count_run(const PsItem* a, int n, bool* desc) {
    *desc = false;
    if (n == 1) return 1;
    int k = 2;
    if (lt(a[1], a[0])) {
        *desc = true;
        for (; k < n; ++k)
            if (!lt(a[k], a[k - 1])) break;
    } else {
        for (; k < n; ++k)
            if (lt(a[k], a[k - 1])) break;
    }
    return k;
}

PL_DEV void binarysort(PsItem* a, int n, int start) {
    if (start == 0) start = 1;
    for (; start < n; ++start) {
        int l = 0, r = start;
        const PsItem pivot = a[start];
        do {
            const int p = l + ((r - l) >> 1);
            if (lt(pivot, a[p])) r = p;
            else l = p + 1;
        } while (l < r);
        for (int p = start; p > l; --p) a[p] = a[p - 1];
        a[l] = pivot;
    }
}

PL_DEV int gallop_left(const PsItem key, const PsItem* a, int n, int hint) {
    int ofs = 1, lastofs = 0, maxofs;
    const PsItem* h = a + hint;
    if (lt(*h, key)) {
        maxofs = n - hint;
        while (ofs < maxofs) {
            if (lt(h[ofs], key)) {
                lastofs = ofs;
                ofs = (ofs << 1) + 1;
            } else {
                break;
            }
        }
        if (ofs > maxofs) ofs = maxofs;
        lastofs += hint;
        ofs += hint;
    } else {
        maxofs = hint + 1;
        while (ofs < maxofs) {
            if (lt(*(h - ofs), key)) break;
            lastofs = ofs;
            ofs = (ofs << 1) + 1;
        }
        if (ofs > maxofs) ofs = maxofs;
        const int k = lastofs;
        lastofs = hint - ofs;
        ofs = hint - k;
    }
    ++lastofs;
    while (lastofs < ofs) {
        const int m = lastofs + ((ofs - lastofs) >> 1);
        if (lt(a[m], key)) lastofs = m + 1;
        else ofs = m;
    }
    return ofs;
}

PL_DEV int gallop_right(const PsItem key, const PsItem* a, int n, int hint) {
    int ofs = 1, lastofs = 0, maxofs;
    const PsItem* h = a + hint;
    if (lt(key, *h)) {
        maxofs = hint + 1;
        while (ofs < maxofs) {
            if (lt(key, *(h - ofs))) {
                lastofs = ofs;
                ofs = (ofs << 1) + 1;
            } else {
                break;
            }
        }
        if (ofs > maxofs) ofs = maxofs;
        const int k = lastofs;
        lastofs = hint - ofs;
        ofs = hint - k;
    } else {
        maxofs = n - hint;
        while (ofs < maxofs) {
            if (lt(key, h[ofs])) break;
            lastofs = ofs;
            ofs = (ofs << 1) + 1;
        }
        if (ofs > maxofs) ofs = maxofs;
        lastofs += hint;
        ofs += hint;
    }
    ++lastofs;
    while (lastofs < ofs) {
        const int m = lastofs + ((ofs - lastofs) >> 1);
        if (lt(key, a[m])) ofs = m;
        else lastofs = m + 1;
    }
    return ofs;
}

struct State {
    PsItem* a;
    PsItem* tmp;
    int min_gallop;
    int n;
    int base[kMaxPending], len[kMaxPending];
};

// na <= nb; run A = a[pa, pa+na) copied to tmp, run B = a[pb, pb+nb), pb = pa + na
PL_DEV void merge_lo(State& s, int pa, int na, int pb, int nb) {
    PsItem* dest = s.a + pa;
    PsItem* A = s.tmp;
    copy_fwd(A, s.a + pa, na);
    PsItem* B = s.a + pb;
    int ia = 0, ib = 0, min_gallop;
    *dest++ = B[ib++];
    --nb;
    if (nb == 0) goto succeed;
    if (na == 1) goto copyb;
    min_gallop = s.min_gallop;
    for (;;) {
        int acount = 0, bcount = 0;
        for (;;) {
            if (lt(B[ib], A[ia])) {
                *dest++ = B[ib++];
                ++bcount;
                acount = 0;
                --nb;
                if (nb == 0) goto succeed;
                if (bcount >= min_gallop) break;
            } else {
                *dest++ = A[ia++];
                ++acount;
                bcount = 0;
                --na;
                if (na == 1) goto copyb;
                if (acount >= min_gallop) break;
            }
        }
        ++min_gallop;
        do {
            min_gallop -= min_gallop > 1;
            s.min_gallop = min_gallop;
            int k = gallop_right(B[ib], A + ia, na, 0);
            acount = k;
            if (k) {
                copy_fwd(dest, A + ia, k);
                dest += k;
                ia += k;
                na -= k;
                if (na == 1) goto copyb;
                if (na == 0) goto succeed;  // only with an inconsistent comparison (NaN)
            }
            *dest++ = B[ib++];
            --nb;
            if (nb == 0) goto succeed;
            k = gallop_left(A[ia], B + ib, nb, 0);
            bcount = k;
            if (k) {
                copy_fwd(dest, B + ib, k);  // dest trails B: forward copy is a memmove
                dest += k;
                ib += k;
                nb -= k;
                if (nb == 0) goto succeed;
            }
            *dest++ = A[ia++];
            --na;
            if (na == 1) goto copyb;
        } while (acount >= kMinGallop || bcount >= kMinGallop);
        ++min_gallop;
        s.min_gallop = min_gallop;
    }
succeed:
    if (na) copy_fwd(dest, A + ia, na);
    return;
copyb:
    copy_fwd(dest, B + ib, nb);
    dest[nb] = A[ia];
}

// na > nb; run B copied to tmp, merged from the right
PL_DEV void merge_hi(State& s, int pa, int na, int pb, int nb) {
    PsItem* const d = s.a;
    const PsItem* basea = s.a + pa;
    PsItem* baseb = s.tmp;
    copy_fwd(baseb, s.a + pb, nb);
    int dest = pb + nb - 1;
    int ia = na - 1, ib = nb - 1, min_gallop;
    d[dest--] = basea[ia--];
    --na;
    if (na == 0) goto succeed;
    if (nb == 1) goto copya;
    min_gallop = s.min_gallop;
    for (;;) {
        int acount = 0, bcount = 0;
        for (;;) {
            if (lt(baseb[ib], basea[ia])) {
                d[dest--] = basea[ia--];
                ++acount;
                bcount = 0;
                --na;
                if (na == 0) goto succeed;
                if (acount >= min_gallop) break;
            } else {
                d[dest--] = baseb[ib--];
                ++bcount;
                acount = 0;
                --nb;
                if (nb == 1) goto copya;
                if (bcount >= min_gallop) break;
            }
        }
        ++min_gallop;
        do {
            min_gallop -= min_gallop > 1;
            s.min_gallop = min_gallop;
            int k = gallop_right(baseb[ib], basea, na, na - 1);
            k = na - k;
            acount = k;
            if (k) {
                dest -= k;
                ia -= k;
                copy_bwd(d + dest + 1, basea + ia + 1, k);  // moving right within a
                na -= k;
                if (na == 0) goto succeed;
            }
            d[dest--] = baseb[ib--];
            --nb;
            if (nb == 1) goto copya;
            if (nb == 0) goto succeed;  // only with an inconsistent comparison (NaN)
            k = gallop_left(basea[ia], baseb, nb, nb - 1);
            k = nb - k;
            bcount = k;
            if (k) {
                dest -= k;
                ib -= k;
                copy_fwd(d + dest + 1, baseb + ib + 1, k);
                nb -= k;
                if (nb == 1) goto copya;
                if (nb == 0) goto succeed;
            }
            d[dest--] = basea[ia--];
            --na;
            if (na == 0) goto succeed;
        } while (acount >= kMinGallop || bcount >= kMinGallop);
        ++min_gallop;
        s.min_gallop = min_gallop;
    }
succeed:
    if (nb) copy_fwd(d + dest - (nb - 1), baseb, nb);
    return;
copya:
    dest -= na;
    ia -= na;
    copy_bwd(d + dest + 1, basea + ia + 1, na);
    d[dest] = baseb[ib];
}

PL_DEV void merge_at(State& s, int i) {
    int pa = s.base[i], na = s.len[i];
    const int pb = s.base[i + 1];
    int nb = s.len[i + 1];
    s.len[i] = na + nb;
    if (i == s.n - 3) {
        s.base[i + 1] = s.base[i + 2];
        s.len[i + 1] = s.len[i + 2];
    }
    --s.n;
    const int k = gallop_right(s.a[pb], s.a + pa, na, 0);
    pa += k;
    na -= k;
    if (na == 0) return;
    nb = gallop_left(s.a[pa + na - 1], s.a + pb, nb, nb - 1);
    if (nb <= 0) return;
    if (na <= nb) merge_lo(s, pa, na, pb, nb);
    else merge_hi(s, pa, na, pb, nb);
}

PL_DEV void merge_collapse(State& s) {
    while (s.n > 1) {
        int n = s.n - 2;
        if ((n > 0 && s.len[n - 1] <= s.len[n] + s.len[n + 1]) ||
            (n > 1 && s.len[n - 2] <= s.len[n - 1] + s.len[n])) {
            if (s.len[n - 1] < s.len[n + 1]) --n;
            merge_at(s, n);
        } else if (s.len[n] <= s.len[n + 1]) {
            merge_at(s, n);
        } else {
            break;
        }
    }
}

PL_DEV void merge_force_collapse(State& s) {
    while (s.n > 1) {
        int n = s.n - 2;
        if (n > 0 && s.len[n - 1] < s.len[n + 1]) --n;
        merge_at(s, n);
    }
}

}  // namespace pysort

// list.sort(key=k, reverse=True) of a[0..n); tmp holds n/2 + 1 items.
PL_DEV void py_sort_desc(PsItem* a, int n, PsItem* tmp) {
    using namespace pysort;
    reverse(a, n);
    if (n >= 2) {
        State s;
        s.a = a;
        s.tmp = tmp;
        s.min_gallop = kMinGallop;
        s.n = 0;
        const int mr = minrun(n);
        int lo = 0, rem = n;
        do {
            bool desc;
            int k = count_run(a + lo, rem, &desc);
            if (desc) reverse(a + lo, k);
            if (k < mr) {
                const int force = rem <= mr ? rem : mr;
                binarysort(a + lo, force, k);
                k = force;
            }
            s.base[s.n] = lo;
            s.len[s.n] = k;
            ++s.n;
            merge_collapse(s);
            lo += k;
            rem -= k;
        } while (rem);
        merge_force_collapse(s);
    }
    reverse(a, n);
}

}  // namespace pl
