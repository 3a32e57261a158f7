/*
 * oracle/pysort.h -- TEST INFRASTRUCTURE ONLY (included by refcpu.c).
 *
 * The order in which CPython 3.10's list.sort(key=..., reverse=True) leaves a
 * list, restated for keys compared with `<` only (Objects/listobject.c,
 * listsort / count_run / binarysort / merge_collapse / merge_at / gallop_left /
 * gallop_right / merge_lo / merge_hi, MIN_GALLOP = 7).  The reference sorts its
 * SCL candidates this way (src/polar/decoder.py:307): for finite keys the result
 * is the stable descending order, but NaN path metrics (+-inf LLRs meeting in a
 * g, decoder.py:417) compare false both ways and the result is whatever this
 * algorithm produces -- so it is restated step by step, including the branches
 * CPython reaches only with an inconsistent comparison.  Pinned against the
 * interpreter itself (tests/test_oracle_golden.py::test_pysort_matches_cpython)
 * and against reference SCL decodes of frames with NaN metrics
 * (tests/golden/polar_nan.npz).
 *
 * reverse=True: CPython reverses the list, sorts it ascending with its stable
 * algorithm, and reverses the result (listobject.c list_sort_impl).
 */
#ifndef ORC_PYSORT_H
#define ORC_PYSORT_H

#include <string.h>

typedef struct { double k; int v; } ps_item;

#define PS_LT(a, b) ((a).k < (b).k)
#define PS_MIN_GALLOP 7
#define PS_MAX_PENDING 85

typedef struct { int base, len; } ps_run;
typedef struct {
    ps_item* a;
    ps_item* tmp;
    int min_gallop;
    int n;
    ps_run pending[PS_MAX_PENDING];
} ps_state;

static void ps_reverse(ps_item* a, int n) {
    for (int i = 0, j = n - 1; i < j; i++, j--) { ps_item t = a[i]; a[i] = a[j]; a[j] = t; }
}

static int ps_minrun(int n) {
    int r = 0;
    while (n >= 64) { r |= n & 1; n >>= 1; }
    return n + r;
}

/* count_run: length of the run at a[0..n), *desc = 1 for a strictly descending run */
static int ps_count_run(const ps_item* a, int n, int* desc) {
    *desc = 0;
    if (n == 1) return 1;
    int k = 2;
    if (PS_LT(a[1], a[0])) {
        *desc = 1;
        for (; k < n; k++) if (!PS_LT(a[k], a[k - 1])) break;
    } else {
        for (; k < n; k++) if (PS_LT(a[k], a[k - 1])) break;
    }
    return k;
}

/* binarysort: a[0..start) sorted; insert a[start..n) one by one */
static void ps_binarysort(ps_item* a, int n, int start) {
    if (start == 0) start = 1;
    for (; start < n; start++) {
        int l = 0, r = start;
        const ps_item pivot = a[start];
        do {
            const int p = l + ((r - l) >> 1);
            if (PS_LT(pivot, a[p])) r = p; else l = p + 1;
        } while (l < r);
        for (int p = start; p > l; p--) a[p] = a[p - 1];
        a[l] = pivot;
    }
}

/* gallop_left: k such that a[k-1] < key <= a[k], starting near hint */
static int ps_gallop_left(ps_item key, const ps_item* a, int n, int hint) {
    int ofs = 1, lastofs = 0, maxofs;
    const ps_item* h = a + hint;
    if (PS_LT(*h, key)) {
        maxofs = n - hint;
        while (ofs < maxofs) {
            if (PS_LT(h[ofs], key)) { lastofs = ofs; ofs = (ofs << 1) + 1; }
            else break;
        }
        if (ofs > maxofs) ofs = maxofs;
        lastofs += hint;
        ofs += hint;
    } else {
        maxofs = hint + 1;
        while (ofs < maxofs) {
            if (PS_LT(*(h - ofs), key)) break;
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
        if (PS_LT(a[m], key)) lastofs = m + 1; else ofs = m;
    }
    return ofs;
}

/* gallop_right: k such that a[k-1] <= key < a[k] */
static int ps_gallop_right(ps_item key, const ps_item* a, int n, int hint) {
    int ofs = 1, lastofs = 0, maxofs;
    const ps_item* h = a + hint;
    if (PS_LT(key, *h)) {
        maxofs = hint + 1;
        while (ofs < maxofs) {
            if (PS_LT(key, *(h - ofs))) { lastofs = ofs; ofs = (ofs << 1) + 1; }
            else break;
        }
        if (ofs > maxofs) ofs = maxofs;
        const int k = lastofs;
        lastofs = hint - ofs;
        ofs = hint - k;
    } else {
        maxofs = n - hint;
        while (ofs < maxofs) {
            if (PS_LT(key, h[ofs])) break;
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
        if (PS_LT(key, a[m])) ofs = m; else lastofs = m + 1;
    }
    return ofs;
}

/* merge_lo: na <= nb, a = s->a + pa, b = s->a + pb = a + na */
static void ps_merge_lo(ps_state* s, int pa, int na, int pb, int nb) {
    ps_item* dest = s->a + pa;
    ps_item* A = s->tmp;
    memcpy(A, s->a + pa, sizeof(ps_item) * na);
    ps_item* B = s->a + pb;
    int ia = 0, ib = 0, min_gallop;
    *dest++ = B[ib++];
    --nb;
    if (nb == 0) goto succeed;
    if (na == 1) goto copyb;
    min_gallop = s->min_gallop;
    for (;;) {
        int acount = 0, bcount = 0;
        for (;;) {
            if (PS_LT(B[ib], A[ia])) {
                *dest++ = B[ib++];
                ++bcount; acount = 0; --nb;
                if (nb == 0) goto succeed;
                if (bcount >= min_gallop) break;
            } else {
                *dest++ = A[ia++];
                ++acount; bcount = 0; --na;
                if (na == 1) goto copyb;
                if (acount >= min_gallop) break;
            }
        }
        ++min_gallop;
        do {
            int k;
            min_gallop -= min_gallop > 1;
            s->min_gallop = min_gallop;
            k = ps_gallop_right(B[ib], A + ia, na, 0);
            acount = k;
            if (k) {
                memcpy(dest, A + ia, sizeof(ps_item) * k);
                dest += k; ia += k; na -= k;
                if (na == 1) goto copyb;
                if (na == 0) goto succeed;
            }
            *dest++ = B[ib++];
            --nb;
            if (nb == 0) goto succeed;
            k = ps_gallop_left(A[ia], B + ib, nb, 0);
            bcount = k;
            if (k) {
                memmove(dest, B + ib, sizeof(ps_item) * k);
                dest += k; ib += k; nb -= k;
                if (nb == 0) goto succeed;
            }
            *dest++ = A[ia++];
            --na;
            if (na == 1) goto copyb;
        } while (acount >= PS_MIN_GALLOP || bcount >= PS_MIN_GALLOP);
        ++min_gallop;
        s->min_gallop = min_gallop;
    }
succeed:
    if (na) memcpy(dest, A + ia, sizeof(ps_item) * na);
    return;
copyb:
    memmove(dest, B + ib, sizeof(ps_item) * nb);
    dest[nb] = A[ia];
}

/* merge_hi: na > nb */
static void ps_merge_hi(ps_state* s, int pa, int na, int pb, int nb) {
    ps_item* basea = s->a + pa;
    ps_item* baseb = s->tmp;
    memcpy(baseb, s->a + pb, sizeof(ps_item) * nb);
    int dest = pb + nb - 1;  /* index into s->a */
    int ia = na - 1, ib = nb - 1, min_gallop;
    ps_item* d = s->a;
    d[dest--] = basea[ia--];
    --na;
    if (na == 0) goto succeed;
    if (nb == 1) goto copya;
    min_gallop = s->min_gallop;
    for (;;) {
        int acount = 0, bcount = 0;
        for (;;) {
            if (PS_LT(baseb[ib], basea[ia])) {
                d[dest--] = basea[ia--];
                ++acount; bcount = 0; --na;
                if (na == 0) goto succeed;
                if (acount >= min_gallop) break;
            } else {
                d[dest--] = baseb[ib--];
                ++bcount; acount = 0; --nb;
                if (nb == 1) goto copya;
                if (bcount >= min_gallop) break;
            }
        }
        ++min_gallop;
        do {
            int k;
            min_gallop -= min_gallop > 1;
            s->min_gallop = min_gallop;
            k = ps_gallop_right(baseb[ib], basea, na, na - 1);
            k = na - k;
            acount = k;
            if (k) {
                dest -= k;
                ia -= k;
                memmove(d + dest + 1, basea + ia + 1, sizeof(ps_item) * k);
                na -= k;
                if (na == 0) goto succeed;
            }
            d[dest--] = baseb[ib--];
            --nb;
            if (nb == 1) goto copya;
            if (nb == 0) goto succeed;
            k = ps_gallop_left(basea[ia], baseb, nb, nb - 1);
            k = nb - k;
            bcount = k;
            if (k) {
                dest -= k;
                ib -= k;
                memcpy(d + dest + 1, baseb + ib + 1, sizeof(ps_item) * k);
                nb -= k;
                if (nb == 1) goto copya;
                if (nb == 0) goto succeed;
            }
            d[dest--] = basea[ia--];
            --na;
            if (na == 0) goto succeed;
        } while (acount >= PS_MIN_GALLOP || bcount >= PS_MIN_GALLOP);
        ++min_gallop;
        s->min_gallop = min_gallop;
    }
succeed:
    if (nb) memcpy(d + dest - (nb - 1), baseb, sizeof(ps_item) * nb);
    return;
copya:
    dest -= na;
    ia -= na;
    memmove(d + dest + 1, basea + ia + 1, sizeof(ps_item) * na);
    d[dest] = baseb[ib];
}

static void ps_merge_at(ps_state* s, int i) {
    int pa = s->pending[i].base, na = s->pending[i].len;
    int pb = s->pending[i + 1].base, nb = s->pending[i + 1].len;
    s->pending[i].len = na + nb;
    if (i == s->n - 3) s->pending[i + 1] = s->pending[i + 2];
    --s->n;
    /* where does b start in a? */
    const int k = ps_gallop_right(s->a[pb], s->a + pa, na, 0);
    pa += k;
    na -= k;
    if (na == 0) return;
    /* where does a end in b? */
    nb = ps_gallop_left(s->a[pa + na - 1], s->a + pb, nb, nb - 1);
    if (nb <= 0) return;
    if (na <= nb) ps_merge_lo(s, pa, na, pb, nb);
    else ps_merge_hi(s, pa, na, pb, nb);
}

static void ps_merge_collapse(ps_state* s) {
    ps_run* p = s->pending;
    while (s->n > 1) {
        int n = s->n - 2;
        if ((n > 0 && p[n - 1].len <= p[n].len + p[n + 1].len) ||
            (n > 1 && p[n - 2].len <= p[n - 1].len + p[n].len)) {
            if (p[n - 1].len < p[n + 1].len) --n;
            ps_merge_at(s, n);
        } else if (p[n].len <= p[n + 1].len) {
            ps_merge_at(s, n);
        } else {
            break;
        }
    }
}

static void ps_merge_force_collapse(ps_state* s) {
    ps_run* p = s->pending;
    while (s->n > 1) {
        int n = s->n - 2;
        if (n > 0 && p[n - 1].len < p[n + 1].len) --n;
        ps_merge_at(s, n);
    }
}

/* ascending CPython sort of a[0..n) with `<`; tmp holds >= n/2 + 1 items */
static void ps_listsort(ps_item* a, int n, ps_item* tmp) {
    if (n < 2) return;
    ps_state s;
    s.a = a;
    s.tmp = tmp;
    s.min_gallop = PS_MIN_GALLOP;
    s.n = 0;
    const int minrun = ps_minrun(n);
    int lo = 0, rem = n;
    do {
        int desc;
        int k = ps_count_run(a + lo, rem, &desc);
        if (desc) ps_reverse(a + lo, k);
        if (k < minrun) {
            const int force = rem <= minrun ? rem : minrun;
            ps_binarysort(a + lo, force, k);
            k = force;
        }
        s.pending[s.n].base = lo;
        s.pending[s.n].len = k;
        ++s.n;
        ps_merge_collapse(&s);
        lo += k;
        rem -= k;
    } while (rem);
    ps_merge_force_collapse(&s);
}

/* list.sort(key=k, reverse=True) */
static void ps_sort_desc(ps_item* a, int n, ps_item* tmp) {
    ps_reverse(a, n);
    ps_listsort(a, n, tmp);
    ps_reverse(a, n);
}

#endif
