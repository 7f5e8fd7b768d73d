/*
 * ORACLE — test infrastructure only (the checker and the bench's CPU
 * baseline, never the product path).
 *
 * C restatement of the reference's per-family consensus hot path
 * (/root/reference/DuplexUMIConsensusReads.py, ":line" below) over the packed
 * batch layout of include/dcr.h.  It follows the reference step by step:
 * expanded CIGAR lists, a materialised aligned matrix, per-column likelihood
 * products in read order, then the field adjustments.  It shares no code with
 * the HIP path.  Pinned against the reference's golden vectors through
 * tests/test_oracle_c.py (same families as the Python oracle).
 *
 * Build: make -C oracle  (gcc -O2 -ffp-contract=off: no FMA contraction,
 * IEEE binary64 throughout, like the reference's numpy float64 scalars).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dcr.h"

typedef struct {
    int pos;
    int len;              /* kept sequence length                     */
    const uint8_t *seq;   /* first kept base                          */
    const uint8_t *qual;
    uint8_t *ops;         /* expanded cigar (=/X already M), n_ops    */
    int n_ops;
    int mask;             /* apply mask_low_quality_bases' 'N'        */
    int mapq;
} oread;

typedef struct {
    uint8_t status;
    int pos, mapq, len, n_cig, n_de, D, M;
    double E;
} ocore;

/* ------------------------------------------------------------ helpers */
static int expand_ops(const uint32_t *cig, int n, uint8_t **out) {
    int tot = 0;
    for (int i = 0; i < n; ++i) tot += (int)(cig[i] >> 4);
    uint8_t *o = (uint8_t *)malloc(tot > 0 ? tot : 1);
    int k = 0;
    for (int i = 0; i < n; ++i)
        for (uint32_t j = 0; j < (cig[i] >> 4); ++j) o[k++] = (uint8_t)(cig[i] & 15);
    *out = o;
    return tot;
}

static int char_class(uint8_t c) {   /* most_likely_nucleotide classes :591 */
    switch (c) {
    case 'A': case 'a': return 0;
    case 'T': case 't': return 1;
    case 'C': case 'c': return 2;
    case 'G': case 'g': return 3;
    case '+': return 4;
    case '-': return 5;
    case 'N': case 'n': return 6;
    default: return -1;
    }
}

static int is_lower(uint8_t c) { return c >= 'a' && c <= 'z'; }

/* numpy pairwise summation (np.add.reduce of the E vector, :1018) */
static double pairwise(const double *a, int64_t n) {
    if (n < 8) {
        double r = -0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise(a, n2) + pairwise(a + n2, n - n2);
}

static int phred_of(const dcr_params *P, double e, int *overflow) {
    /* :699-709, with the host-tabulated rounding boundaries */
    double pre = (double)P->error_rate_pre_labeling, post = (double)P->error_rate_post_labeling;
    double x = pre * (1.0 - e) + (1.0 - post) * e + pre * e * 4.0 / 5.0;
    if (!(x > 0.0)) return P->max_base_quality;      /* ValueError branch (0, <0, NaN) */
    if (isinf(x)) { *overflow = 1; return 0; }       /* int(-inf): OverflowError */
    int c = 0;
    for (int i = 0; i < P->n_qthresh; ++i) c += (x >= P->qthresh[i]);
    int q = P->max_base_quality - c;
    if (q < 0 || q > 255) *overflow = 1;
    return q;
}

/* ----------------------------------------------------- one consensus */
/* make_consensus_read (:1291-1386) on prepared reads; writes the record's
 * variable-length fields at the given pointers (capacity cap). */
static void consensus(const dcr_params *P, oread *rd, int R, int64_t cap, ocore *oc,
                      uint8_t *oseq, uint8_t *oqual, uint32_t *ocig, uint16_t *od, uint16_t *oe) {
    memset(oc, 0, sizeof(*oc));
    for (int r = 0; r < R; ++r)
        if (rd[r].len == 0) { oc->status = DCR_ST_TYPE_ERROR; return; }   /* list(None) :402 */
    /* reconstruct_alignment :430-547 */
    int min_pos = rd[0].pos, max_pos = rd[0].pos + rd[0].len;
    for (int r = 1; r < R; ++r) {
        if (rd[r].pos < min_pos) min_pos = rd[r].pos;
        if (rd[r].pos + rd[r].len > max_pos) max_pos = rd[r].pos + rd[r].len;
    }
    int T = max_pos - min_pos;
    if (T > cap) { oc->status = 255; return; }
    uint8_t *al = (uint8_t *)malloc((size_t)R * T + 1);
    int16_t *aq = (int16_t *)malloc(sizeof(int16_t) * ((size_t)R * T + 1));
    int *ic = (int *)calloc(R, sizeof(int)), *is = (int *)calloc(R, sizeof(int));
    for (int t = 0; t < T; ++t) {
        int p = min_pos + t, any_ins = 0;
        for (int r = 0; r < R; ++r)
            if (ic[r] < rd[r].n_ops && rd[r].ops[ic[r]] == 1) any_ins = 1;      /* :476-478 */
        for (int r = 0; r < R; ++r) {
            uint8_t *a = &al[(size_t)r * T + t];
            int16_t *q = &aq[(size_t)r * T + t];
            int op = ic[r] < rd[r].n_ops ? rd[r].ops[ic[r]] : 0;
            if (any_ins) {
                if (op == 1) {
                    if (is[r] >= rd[r].len) { oc->status = DCR_ST_INDEX_ERROR; goto done; }
                    uint8_t b = rd[r].seq[is[r]], qq = rd[r].qual[is[r]];
                    if (rd[r].mask && qq < P->min_base_quality) b = 'N';
                    *a = (uint8_t)(b >= 'A' && b <= 'Z' ? b + 32 : b);
                    *q = qq;
                    ic[r]++; is[r]++;
                } else { *a = '+'; *q = DCR_LUT_PLUS; }
            } else if (p < rd[r].pos) { *a = 'N'; *q = 2; }
            else if (is[r] < rd[r].len) {
                if (ic[r] >= rd[r].n_ops) { oc->status = DCR_ST_INDEX_ERROR; goto done; }
                if (rd[r].ops[ic[r]] == 2) { *a = '-'; *q = DCR_LUT_DEL; ic[r]++; }
                else {
                    uint8_t b = rd[r].seq[is[r]], qq = rd[r].qual[is[r]];
                    if (rd[r].mask && qq < P->min_base_quality) b = 'N';
                    *a = b; *q = qq; ic[r]++; is[r]++;
                }
            } else { *a = 'N'; *q = 2; }
        }
    }
    {
        /* call_consensus :625-712 */
        uint8_t *cons = (uint8_t *)malloc(T + 1);
        int *cq = (int *)malloc(sizeof(int) * (T + 1));
        int overflow = 0;
        for (int t = 0; t < T; ++t) {
            double L[6] = {1, 1, 1, 1, 1, 1};
            int has_plus = 0;
            for (int r = 0; r < R; ++r) {
                uint8_t c = al[(size_t)r * T + t];
                int k = char_class(c);
                if (k < 0) { oc->status = DCR_ST_EXIT_BADCHAR; free(cons); free(cq); goto done; }
                if (c == '+') has_plus = 1;
                int li = aq[(size_t)r * T + t];
                double m = P->match[li], mm = P->mismatch[li];
                for (int i = 0; i < 6; ++i) L[i] *= (i == k) ? m : mm;
            }
            double S = L[0] + L[1];
            S = S + L[2]; S = S + L[3]; S = S + L[4]; S = S + L[5];
            int best = 0;
            double pm = L[0] / S;
            for (int i = 0; i < 6; ++i) {
                double pi = L[i] / S;
                if (isnan(pi)) { best = i; pm = pi; break; }
                if (pi > pm) { best = i; pm = pi; }
            }
            uint8_t ch = (uint8_t)"ATCG+-"[best];
            if (has_plus && ch >= 'A' && ch <= 'Z') ch += 32;
            if (pm < P->post_threshold) ch = has_plus ? 'n' : 'N';
            cons[t] = ch;
            cq[t] = phred_of(P, 1.0 - pm, &overflow);
        }
        /* adjust_consensus_fields :745-871 */
        int t5 = 0, t3 = T;
        while (t5 < T && cons[t5] == 'N') t5++;
        while (t3 > 0 && cons[t3 - 1] == 'N') t3--;
        int n = t3 > t5 ? t3 - t5 : 0;
        const uint8_t *cs = cons + t5;
        uint8_t *opl = (uint8_t *)malloc(n + 1);
        int nops = 0;
        for (int i = 0; i < n; ++i) {
            uint8_t c = cs[i];
            if (is_lower(c)) {
                if (i + 1 < n && cs[i + 1] == '-') { opl[nops++] = 0; i++; }
                else opl[nops++] = 1;
            } else if (c == '+') {
            } else if (c == '-') {
                if (i + 1 < n && is_lower(cs[i + 1])) { opl[nops++] = 0; i++; }
                else opl[nops++] = 2;
            } else opl[nops++] = 0;
        }
        if (nops == 0) { oc->status = DCR_ST_INDEX_ERROR; free(opl); free(cons); free(cq); goto done; }
        int nc = 0;
        for (int i = 0; i < nops; ++i) {
            if (nc > 0 && (int)(ocig[nc - 1] & 15) == opl[i]) ocig[nc - 1] += 16;
            else ocig[nc++] = (1u << 4) | opl[i];
        }
        int len = 0;
        for (int i = 0; i < n; ++i) {
            uint8_t c = cs[i];
            if (c == '+' || c == '-') continue;
            oseq[len] = (uint8_t)(c >= 'a' && c <= 'z' ? c - 32 : c);
            oqual[len] = (uint8_t)cq[t5 + i];
            len++;
        }
        /* calculate_depth_and_errors :970-1021 */
        int nde = 0, D = -1, M = 1 << 30;
        double *Et = (double *)malloc(sizeof(double) * (T + 1));
        for (int t = 0; t < T; ++t) {
            if (cons[t] == '+') continue;
            int d = 0, e = 0;
            for (int r = 0; r < R; ++r) {
                uint8_t c = al[(size_t)r * T + t];
                d += !(c == 'N' || c == 'n' || c == '+');
                e += (c != cons[t]);
            }
            od[nde] = (uint16_t)d; oe[nde] = (uint16_t)e;
            Et[nde] = d == 0 ? 1.0 : (double)e / (double)d;
            if (d > D) D = d;
            if (d < M) M = d;
            nde++;
        }
        if (nde == 0) oc->status = DCR_ST_VALUE_ERROR;
        else if (overflow) {
            /* only qualities kept in the record reach pysam (:1383) */
            for (int i = 0; i < n; ++i)
                if (cs[i] != '+' && cs[i] != '-' && (cq[t5 + i] < 0 || cq[t5 + i] > 255))
                    oc->status = DCR_ST_OVERFLOW_ERROR;
        }
        double mean = (0.0 + pairwise(Et, nde)) / (double)nde;
        double y = mean * 1000.0;
        oc->E = nearbyint(y) / 1000.0;
        int64_t msum = 0;
        for (int r = 0; r < R; ++r) msum += rd[r].mapq;
        oc->mapq = (int)(msum / R);
        oc->pos = min_pos + t5;
        oc->len = len;
        oc->n_cig = nc;
        oc->n_de = nde;
        oc->D = D;
        oc->M = M;
        free(Et); free(opl); free(cons); free(cq);
    }
done:
    free(al); free(aq); free(ic); free(is);
}

/* remove_clipping :191-265, mask_low_quality_bases :268-289, trim_3prime_N :292-325 */
static void prep_read(const dcr_params *P, const dcr_batch *in, int i, oread *o, dcr_read_info *inf) {
    const uint32_t *cig = in->cigar + in->cig_off[i];
    int n = in->cig_n[i];
    int sc5 = 0, sc3 = 0, inseq = 0, modified = 0;
    uint32_t *kept = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    int nk = 0;
    for (int j = 0; j < n; ++j) {
        int op = cig[j] & 15, ln = cig[j] >> 4;
        if (op == 5) modified = 1;
        else if (op == 4) { modified = 1; if (!inseq) sc5 = ln; else sc3 = ln; }
        else { inseq = 1; kept[nk++] = cig[j]; }
    }
    int len = in->seq_len[i];
    int start = 0;
    memset(inf, 0, sizeof(*inf));
    if (modified) {
        start = sc5;
        len = len - sc5 - sc3;
        if (len < 0) len = 0;
    } else nk = n, memcpy(kept, cig, sizeof(uint32_t) * n);
    const uint8_t *seq = in->bases + in->seq_off[i] + start;
    const uint8_t *qual = in->quals + in->seq_off[i] + start;
    o->pos = in->read_pos[i];
    o->mapq = in->read_mapq[i];
    o->seq = seq;
    o->qual = qual;
    o->mask = 1;
    o->ops = NULL;
    o->n_ops = 0;
    inf->seq_start = in->seq_off[i] + start;
    if (len <= 0) {
        inf->status = DCR_ST_TYPE_ERROR;   /* empty sequence: enumerate(None) :279 */
        o->len = 0;
        free(kept);
        return;
    }
    int tl = len;
    while (tl > 0 && (seq[tl - 1] == 'N' || qual[tl - 1] < P->min_base_quality)) tl--;
    int k = len - tl;
    uint8_t *ops;
    int nops = expand_ops(kept, nk, &ops);
    nops -= k;
    if (nops <= 0) { inf->status = DCR_ST_INDEX_ERROR; nops = 0; }   /* compress_cigarlist([]) */
    for (int j = 0; j < nops; ++j) if (ops[j] == 7 || ops[j] == 8) ops[j] = 0;
    int has_ins = 0, runs = 0;
    for (int j = 0; j < nops; ++j) {
        has_ins |= ops[j] == 1;
        runs += (j == 0 || ops[j] != ops[j - 1]);
    }
    o->ops = ops;
    o->n_ops = nops;
    o->len = tl;
    inf->len = tl;
    inf->n_cig = runs;
    inf->has_ins = has_ins;
    free(kept);
}

typedef struct {
    const dcr_params *P;
    const dcr_batch *in;
    dcr_out *ss, *ds;
    dcr_read_info *info;
    int f0, f1;
} job;

static void write_core(dcr_out *o, int64_t i, const ocore *c) {
    o->status[i] = c->status;
    o->pos[i] = c->pos; o->mapq[i] = c->mapq; o->len[i] = c->len; o->n_cig[i] = c->n_cig;
    o->n_de[i] = c->n_de; o->D[i] = c->D; o->M[i] = c->M; o->E[i] = c->E;
}

static void run_family(const dcr_params *P, const dcr_batch *in, dcr_out *ss, dcr_out *ds,
                       dcr_read_info *info, int f) {
    ocore sc[4];
    int failed[4];
    for (int k = 0; k < 4; ++k) {
        int s = 4 * f + k, a = in->sub_off[s], b = in->sub_off[s + 1], R = b - a;
        oread *rd = (oread *)calloc(R > 0 ? R : 1, sizeof(oread));
        int pre_fail = 0;
        for (int r = 0; r < R; ++r) {
            dcr_read_info tmp;
            prep_read(P, in, a + r, &rd[r], info ? &info[a + r] : &tmp);
            const int st = info ? info[a + r].status : tmp.status;
            if (st != 0 && !pre_fail) pre_fail = DCR_ST_PREP | st;   /* the first failing read :1272-1283 */
        }
        int64_t o = in->ss_col_off[s], cap = in->ss_col_off[s + 1] - o;
        if (R == 0) { memset(&sc[k], 0, sizeof(ocore)); sc[k].status = DCR_ST_VALUE_ERROR; }   /* min([]) :458 */
        else if (pre_fail) { memset(&sc[k], 0, sizeof(ocore)); sc[k].status = pre_fail; }
        else consensus(P, rd, R, cap, &sc[k], ss->seq + o, ss->qual + o, ss->cigar + o, ss->d + o, ss->e + o);
        write_core(ss, s, &sc[k]);
        failed[k] = sc[k].status != 0;
        for (int r = 0; r < R; ++r) free(rd[r].ops);
        free(rd);
    }
    /* duplex: make_consensus_read([A1, B2]) and ([B1, A2]) :1575-1582 on the
       single-strand consensus records (no preprocessing, no masking) */
    for (int j = 0; j < 2; ++j) {
        int p = 2 * f + j;
        int sa = 4 * f + 2 * j, sb = sa + 1;
        ocore c;
        if (failed[2 * j] || failed[2 * j + 1]) {
            memset(&c, 0, sizeof(c));
            c.status = DCR_ST_UPSTREAM;
        } else {
            oread rd[2];
            int ss_i[2] = {sa, sb};
            for (int r = 0; r < 2; ++r) {
                int s = ss_i[r];
                int64_t o = in->ss_col_off[s];
                rd[r].pos = ss->pos[s];
                rd[r].len = ss->len[s];
                rd[r].seq = ss->seq + o;
                rd[r].qual = ss->qual + o;
                rd[r].mask = 0;
                rd[r].mapq = ss->mapq[s];
                rd[r].n_ops = expand_ops(ss->cigar + o, ss->n_cig[s], &rd[r].ops);
            }
            int64_t o = in->ds_col_off[p], cap = in->ds_col_off[p + 1] - o;
            consensus(P, rd, 2, cap, &c, ds->seq + o, ds->qual + o, ds->cigar + o, ds->d + o, ds->e + o);
            free(rd[0].ops); free(rd[1].ops);
        }
        write_core(ds, p, &c);
    }
}

static void *worker(void *arg) {
    job *j = (job *)arg;
    for (int f = j->f0; f < j->f1; ++f) run_family(j->P, j->in, j->ss, j->ds, j->info, f);
    return NULL;
}

int dcr_oracle_run(const dcr_params *P, const dcr_batch *in, dcr_out *ss, dcr_out *ds,
                   dcr_read_info *info, int n_threads) {
    if (!P || !in || !ss || !ds) return DCR_EARG;
    if (n_threads <= 1 || in->n_fam < 2 * n_threads) {
        for (int f = 0; f < in->n_fam; ++f) run_family(P, in, ss, ds, info, f);
        return DCR_OK;
    }
    pthread_t th[256];
    job jobs[256];
    if (n_threads > 256) n_threads = 256;
    int per = (in->n_fam + n_threads - 1) / n_threads;
    for (int t = 0; t < n_threads; ++t) {
        jobs[t] = (job){P, in, ss, ds, info, t * per, (t + 1) * per < in->n_fam ? (t + 1) * per : in->n_fam};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    return DCR_OK;
}
