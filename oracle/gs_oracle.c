/*
 * gs_oracle.c -- CPU restatement of GeneralSparse's SpMM hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see gs_oracle.h).  Deliberately literal and
 * single-threaded: each function walks the data the way the cited reference
 * transform does, so that a reviewer can check it line by line against the
 * reference.  Reference defects are reproduced where they change the plan
 * arrays and guarded (error return) where the reference would crash.
 */
#include "gs_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define PADDING_RATE_UP_BOUND 4 /* global_config.json.bak:25 */

/* ------------------------------------------------------------------ */
/* named-array set (metadata_set.cc:147-151, :255-331)                 */
/* ------------------------------------------------------------------ */

static int fail(or_set *s, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(s->err, sizeof(s->err), fmt, ap);
    va_end(ap);
    return -1;
}

static void mkkey(char *out, const char *pos, const char *name, int sub) {
    snprintf(out, OR_NAME_LEN, "%s_%s_%d", pos, name, sub);
}

or_array *or_find(or_set *s, const char *key) {
    for (int i = 0; i < s->n; i++)
        if (strcmp(s->a[i].key, key) == 0) return &s->a[i];
    return NULL;
}

static or_array *get(or_set *s, const char *pos, const char *name, int sub) {
    char k[OR_NAME_LEN];
    mkkey(k, pos, name, sub);
    return or_find(s, k);
}

static int exists(or_set *s, const char *pos, const char *name, int sub) {
    return get(s, pos, name, sub) != NULL;
}

static void drop(or_set *s, const char *pos, const char *name, int sub) {
    char k[OR_NAME_LEN];
    mkkey(k, pos, name, sub);
    for (int i = 0; i < s->n; i++) {
        if (strcmp(s->a[i].key, k) == 0) {
            free(s->a[i].u);
            free(s->a[i].f);
            s->a[i] = s->a[s->n - 1];
            s->n--;
            return;
        }
    }
}

/* add_element: takes ownership of data */
static or_array *put_u(or_set *s, const char *pos, const char *name, int sub,
                       uint64_t *data, uint64_t len) {
    drop(s, pos, name, sub);
    if (s->n >= OR_MAX_ARRAYS) abort(); /* the set's fixed capacity */
    or_array *a = &s->a[s->n++];
    memset(a, 0, sizeof(*a));
    mkkey(a->key, pos, name, sub);
    a->len = len;
    a->u = data;
    return a;
}

static or_array *put_f(or_set *s, const char *pos, const char *name, int sub,
                       double *data, uint64_t len) {
    drop(s, pos, name, sub);
    if (s->n >= OR_MAX_ARRAYS) abort(); /* the set's fixed capacity */
    or_array *a = &s->a[s->n++];
    memset(a, 0, sizeof(*a));
    mkkey(a->key, pos, name, sub);
    a->len = len;
    a->is_float = 1;
    a->f = data;
    return a;
}

static or_array *put_scalar(or_set *s, const char *pos, const char *name, int sub,
                            uint64_t v) {
    uint64_t *d = (uint64_t *)malloc(sizeof(uint64_t));
    d[0] = v;
    return put_u(s, pos, name, sub, d, 1);
}

static uint64_t scalar(or_set *s, const char *pos, const char *name, int sub) {
    or_array *a = get(s, pos, name, sub);
    return a ? a->u[0] : 0;
}

void or_set_free(or_set *s) {
    for (int i = 0; i < s->n; i++) {
        free(s->a[i].u);
        free(s->a[i].f);
    }
    s->n = 0;
}

int or_count(const or_set *s) { return s->n; }
const char *or_key(const or_set *s, int i) { return s->a[i].key; }
uint64_t or_len(const or_set *s, int i) { return s->a[i].len; }
int or_is_float(const or_set *s, int i) { return s->a[i].is_float; }
const uint64_t *or_u(const or_set *s, int i) { return s->a[i].u; }
const double *or_f(const or_set *s, int i) { return s->a[i].f; }
const char *or_error(const or_set *s) { return s->err; }

static uint64_t *dup_u(const uint64_t *p, uint64_t n) {
    uint64_t *d = (uint64_t *)malloc((n ? n : 1) * sizeof(uint64_t));
    if (n) memcpy(d, p, n * sizeof(uint64_t));
    return d;
}

/* growable u64 / f64 vectors */
typedef struct { uint64_t *p; uint64_t n, cap; } vu;
static void vu_push(vu *v, uint64_t x) {
    if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 16; v->p = (uint64_t *)realloc(v->p, v->cap * 8); }
    v->p[v->n++] = x;
}

/* ------------------------------------------------------------------ */
/* A1: .mtx reader -- struct.cc:49-261                                  */
/* ------------------------------------------------------------------ */

int or_read_mtx(const char *path, int ones_values, or_coo *out) {
    memset(out, 0, sizeof(*out));
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char buf[1024];
    int first = 1;
    vu rows = {0}, cols = {0};
    float *vals = NULL;
    uint64_t vcap = 0;
    while (fgets(buf, sizeof(buf), f)) {
        size_t L = strlen(buf);
        while (L && (buf[L - 1] == '\n' || buf[L - 1] == '\r')) buf[--L] = 0;
        /* struct.cc:97: skip empty lines, lines starting with whitespace or '%' */
        if (L == 0 || buf[0] == ' ' || buf[0] == '\t' || buf[0] == '%') continue;
        char *tok[3] = {0, 0, 0};
        int nt = 0;
        char *p = buf;
        while (nt < 3 && p) { /* split on single spaces (struct.hpp:290) */
            tok[nt++] = p;
            p = strchr(p, ' ');
            if (p) *p++ = 0;
        }
        if (first) { /* struct.cc:104-110: header gives max indices */
            out->max_row_index = (uint64_t)atol(tok[0]) - 1;
            out->max_col_index = (uint64_t)atol(tok[1]) - 1;
            first = 0;
            continue;
        }
        uint64_t r = (uint64_t)atol(tok[0]) - 1; /* struct.cc:114-116 */
        uint64_t c = (uint64_t)atol(tok[1]) - 1;
        float v = tok[2] ? (float)atof(tok[2]) : 1.0f;
        if (rows.n && r < rows.p[rows.n - 1]) { /* struct.cc:120-131 */
            fclose(f);
            free(rows.p); free(cols.p); free(vals);
            return -2;
        }
        vu_push(&rows, r);
        vu_push(&cols, c);
        if (rows.n > vcap) { vcap = vcap ? vcap * 2 : 16; vals = (float *)realloc(vals, vcap * sizeof(float)); }
        vals[rows.n - 1] = ones_values ? 1.0f : v; /* struct.cc:186-200 */
        if (r > out->max_row_index) out->max_row_index = r; /* struct.cc:203-211 */
        if (c > out->max_col_index) out->max_col_index = c;
    }
    fclose(f);
    if (rows.n == 0) { free(rows.p); free(cols.p); free(vals); return -3; } /* struct.cc:258 */
    out->nnz = rows.n;
    out->row = rows.p;
    out->col = cols.p;
    out->val = vals;
    return 0;
}

void or_coo_free(or_coo *c) {
    free(c->row); free(c->col); free(c->val);
    memset(c, 0, sizeof(*c));
}

/* ------------------------------------------------------------------ */
/* A2: create_init_metadata_set_from_file -- metadata_set.cc:612-707   */
/* ------------------------------------------------------------------ */

int or_init_set(or_set *s, uint64_t n_rows, uint64_t n_cols, uint64_t nnz,
                const uint64_t *row, const uint64_t *col, const float *val) {
    memset(s, 0, sizeof(*s));
    if (nnz == 0) return fail(s, "empty matrix (struct.cc:258)");
    uint64_t max_row = n_rows - 1, max_col = n_cols - 1;
    for (uint64_t i = 0; i < nnz; i++) {
        if (i && row[i] < row[i - 1]) return fail(s, "rows not sorted (struct.cc:125)");
        if (row[i] > max_row) max_row = row[i];
        if (col[i] > max_col) max_col = col[i];
    }
    put_scalar(s, "GLOBAL_META", "origin_row_num", -1, max_row + 1);
    put_scalar(s, "GLOBAL_META", "origin_col_num", -1, max_col + 1);
    put_scalar(s, "GLOBAL_META", "origin_nnz_num", -1, nnz);
    put_scalar(s, "GLOBAL_META", "begin_row_index", 0, 0);
    put_scalar(s, "GLOBAL_META", "begin_col_index", 0, 0);
    put_scalar(s, "GLOBAL_META", "end_row_index", 0, max_row);
    put_scalar(s, "GLOBAL_META", "end_col_index", 0, max_col);
    put_u(s, "GLOBAL_META", "nz_row_indices", 0, dup_u(row, nnz), nnz);
    put_u(s, "GLOBAL_META", "nz_col_indices", 0, dup_u(col, nnz), nnz);
    double *v = (double *)malloc(nnz * sizeof(double));
    for (uint64_t i = 0; i < nnz; i++) v[i] = (double)val[i];
    put_f(s, "GLOBAL_META", "nz_vals", 0, v, nnz);
    return 0;
}

/* get_nnz_of_each_row_in_spec_range -- data_transform_common.cc:7-48 */
static uint64_t *row_nnz(const uint64_t *row, uint64_t nnz, uint64_t row_num) {
    uint64_t *cnt = (uint64_t *)calloc(row_num ? row_num : 1, sizeof(uint64_t));
    for (uint64_t i = 0; i < nnz; i++) cnt[row[i]]++;
    return cnt;
}

/* the "real end row" rule repeated in every transform, e.g.
 * get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction.cc:60-66 */
static uint64_t row_num_of(or_set *s) {
    uint64_t b = scalar(s, "GLOBAL_META", "begin_row_index", 0);
    uint64_t e = scalar(s, "GLOBAL_META", "end_row_index", 0);
    or_array *r = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t real = b + r->u[r->len - 1];
    if (e < real) e = real;
    return e - b + 1;
}

/* ------------------------------------------------------------------ */
/* A3/A4: sort_operator -- operator/sort_operator.cc:70-108             */
/* ------------------------------------------------------------------ */

int or_sort_operator(or_set *s) {
    if (exists(s, "GLOBAL_META", "original_nz_row_indices", 0))
        return fail(s, "already sorted (sort_operator.cc:55-65)");
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t nnz = R->len;
    /* get_row_order_by_length.cc:36-55: row range incl. empty rows */
    uint64_t minr = scalar(s, "GLOBAL_META", "begin_row_index", 0);
    uint64_t maxr = scalar(s, "GLOBAL_META", "end_row_index", 0);
    uint64_t real_max = R->u[nnz - 1];
    if (real_max > maxr - minr) maxr = minr + real_max;
    uint64_t nrow = maxr - minr + 1;
    uint64_t *cnt = row_nnz(R->u, nnz, nrow);
    uint64_t maxlen = 0;
    for (uint64_t i = 0; i < nrow; i++) if (cnt[i] > maxlen) maxlen = cnt[i];
    /* get_row_order_by_length.cc:67-110: buckets by length, visited from
     * the longest; inside a bucket rows keep ascending order */
    uint64_t *bstart = (uint64_t *)calloc(maxlen + 2, sizeof(uint64_t));
    for (uint64_t i = 0; i < nrow; i++) bstart[cnt[i]]++;
    /* offsets in descending length order */
    uint64_t acc = 0;
    for (int64_t L = (int64_t)maxlen; L >= 0; L--) {
        uint64_t c = bstart[L];
        bstart[L] = acc;
        acc += c;
    }
    uint64_t *order = (uint64_t *)malloc(nrow * sizeof(uint64_t));
    for (uint64_t i = 0; i < nrow; i++) order[bstart[cnt[i]]++] = i;
    free(bstart);
    put_u(s, "GLOBAL_META", "original_nz_row_indices", 0, order, nrow);

    /* reorder_val/col/row_by_index: regroup COO in the new row order,
     * keeping the within-row order (reorder_col_by_index.cc:55-120) */
    uint64_t *start = (uint64_t *)malloc((nrow + 1) * sizeof(uint64_t));
    start[0] = 0;
    for (uint64_t i = 0; i < nrow; i++) start[i + 1] = start[i] + cnt[i];
    /* reorder_col_by_index.cc:82-93 asserts non-decreasing cols in a row */
    for (uint64_t i = 1; i < nnz; i++)
        if (R->u[i] == R->u[i - 1] && C->u[i] < C->u[i - 1]) {
            free(start); free(cnt);
            return fail(s, "cols not sorted within row (reorder_col_by_index.cc:88)");
        }
    uint64_t *nr = (uint64_t *)malloc(nnz * 8), *nc = (uint64_t *)malloc(nnz * 8);
    double *nv = (double *)malloc(nnz * 8);
    uint64_t p = 0;
    for (uint64_t newr = 0; newr < nrow; newr++) {
        uint64_t old = order[newr];
        for (uint64_t k = start[old]; k < start[old + 1]; k++) {
            nr[p] = newr;
            nc[p] = C->u[k];
            nv[p] = V->f[k];
            p++;
        }
    }
    free(start); free(cnt);
    put_f(s, "GLOBAL_META", "nz_vals", 0, nv, nnz);
    put_u(s, "GLOBAL_META", "nz_col_indices", 0, nc, nnz);
    put_u(s, "GLOBAL_META", "nz_row_indices", 0, nr, nnz);
    /* remove_empty_row_in_end_of_sub_matrix.cc:13-70 */
    uint64_t b = scalar(s, "GLOBAL_META", "begin_row_index", 0);
    uint64_t e = scalar(s, "GLOBAL_META", "end_row_index", 0);
    uint64_t last = nr[nnz - 1];
    if (last < e - b) put_scalar(s, "GLOBAL_META", "end_row_index", 0, b + last);
    return 0;
}

/* ------------------------------------------------------------------ */
/* empty_row_pad_operator (operator/empty_row_pad_operator.cc:30-147)  */
/* + modify_{col,val,row}_*_by_empty_pad_in_submatrix.cc:15-110         */
/* ------------------------------------------------------------------ */

int or_empty_row_pad(or_set *s) {
    /* is_valid_according_to_operator (:25-55): not after sort_operator; the canned
     * sequences here never run it twice or after a distributing operator */
    if (exists(s, "GLOBAL_META", "original_nz_row_indices", 0))
        return fail(s, "empty_row_pad after sort_operator (empty_row_pad_operator.cc:37-52)");
    for (int i = 0; i < s->n; i++)
        if (!strncmp(s->a[i].key, "THREAD_META", 11) || !strncmp(s->a[i].key, "WARP_META", 9) ||
            !strncmp(s->a[i].key, "TBLOCK_META", 11))
            return fail(s, "empty_row_pad with blocking metadata (empty_row_pad_operator.cc:117-121)");
    if (exists(s, "GLOBAL_META", "nz_col_indices_after_interlance_storage", 0))
        return fail(s, "empty_row_pad after interleaving (empty_row_pad_operator.cc:106-112)");
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t nnz = R->len;
    /* :82-95: the row range grows to the largest stored row */
    uint64_t b = scalar(s, "GLOBAL_META", "begin_row_index", 0);
    uint64_t e = scalar(s, "GLOBAL_META", "end_row_index", 0);
    if (R->u[nnz - 1] > e - b) e = b + R->u[nnz - 1];
    uint64_t rn = e - b + 1;
    uint64_t *cnt = row_nnz(R->u, nnz, rn), zeros = 0;
    for (uint64_t r = 0; r < rn; r++) zeros += cnt[r] == 0;
    free(cnt);
    if (!zeros) return fail(s, "no empty row (empty_row_pad_operator.cc:124)");
    /* padding_rate_valid_empty_padding (data_transform_common.cc:600-643) */
    if ((double)(nnz + zeros) / (double)nnz >= PADDING_RATE_UP_BOUND)
        return fail(s, "empty padding rate %.3f >= %d", (double)(nnz + zeros) / nnz, PADDING_RATE_UP_BOUND);
    /* the three transforms: a nonzero whose next nonzero (rn for the last) lies more than
     * one row further is followed by one entry per skipped row (that row, its column,
     * value 0); the walk starts at the first nonzero, so leading empty rows stay empty */
    vu nr = {0}, nc = {0};
    uint64_t fcap = nnz + zeros + 1, fn = 0;
    double *nv = (double *)malloc(fcap * sizeof(double));
    int padded = 0;
    for (uint64_t i = 0; i < nnz; i++) {
        uint64_t r = R->u[i], nxt = i + 1 == nnz ? rn : R->u[i + 1];
        if (nxt == r || nxt == r + 1) {
            vu_push(&nr, r); vu_push(&nc, C->u[i]); nv[fn++] = V->f[i];
            continue;
        }
        double v = V->f[i];
        for (uint64_t id = r; id < nxt; id++) { /* :63-72 (nothing when nxt < r) */
            if (fn == fcap) { fcap *= 2; nv = (double *)realloc(nv, fcap * sizeof(double)); }
            vu_push(&nr, id); vu_push(&nc, C->u[i]); nv[fn++] = v;
            v = 0.0;
            if (id > r) padded = 1;
        }
    }
    if (!padded) { free(nr.p); free(nc.p); free(nv); return 0; }
    put_u(s, "GLOBAL_META", "nz_col_indices", 0, nc.p, nc.n);
    put_f(s, "GLOBAL_META", "nz_vals", 0, nv, fn);
    put_u(s, "GLOBAL_META", "nz_row_indices", 0, nr.p, nr.n);
    return 0;
}

/* ------------------------------------------------------------------ */
/* A6: modify_{col,val,row}_by_col_pad_in_sub_matrix                    */
/*     modify_col_indices_by_col_pad_in_sub_matrix.cc:15-160            */
/* ------------------------------------------------------------------ */

static int col_pad(or_set *s, int mult) {
    if (mult < 2) return fail(s, "col pad multiple < 2 (modify_col...:26)");
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t nnz = R->len, row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, nnz, row_num);
    uint64_t after = nnz;
    for (uint64_t r = 0; r < row_num; r++)
        if (cnt[r] % mult) after += (cnt[r] / mult + 1) * mult - cnt[r];
    if ((double)after / (double)nnz >= PADDING_RATE_UP_BOUND) { /* :103-110 */
        free(cnt);
        return fail(s, "padding rate %.3f >= %d", (double)after / nnz, PADDING_RATE_UP_BOUND);
    }
    if (after == nnz) { free(cnt); return 0; } /* is_padded == false: arrays untouched */
    uint64_t *nr = (uint64_t *)malloc(after * 8), *nc = (uint64_t *)malloc(after * 8);
    double *nv = (double *)malloc(after * 8);
    uint64_t p = 0, q = 0;
    for (uint64_t r = 0; r < row_num; r++) {
        for (uint64_t k = 0; k < cnt[r]; k++, q++) {
            nr[p] = R->u[q]; nc[p] = C->u[q]; nv[p] = V->f[q]; p++;
        }
        if (cnt[r] % mult) {
            uint64_t target = (cnt[r] / mult + 1) * mult;
            uint64_t lastc = nc[p - 1], lastr = nr[p - 1];
            for (uint64_t k = cnt[r]; k < target; k++) { /* :113-116, vals :114 */
                nr[p] = lastr; nc[p] = lastc; nv[p] = 0.0; p++;
            }
        }
    }
    free(cnt);
    put_u(s, "GLOBAL_META", "nz_col_indices", 0, nc, after);
    put_f(s, "GLOBAL_META", "nz_vals", 0, nv, after);
    put_u(s, "GLOBAL_META", "nz_row_indices", 0, nr, after);
    return 0;
}

/* modify_{col,vals,row}_*_by_row_pad_in_sub_matrix.cc: the recorded row range (end - begin + 1)
 * up to a multiple, one entry per added row appended (row = row_num + i, the last column, 0) */
static int row_pad(or_set *s, int mult) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t nnz = R->len;
    uint64_t rn = scalar(s, "GLOBAL_META", "end_row_index", 0) - scalar(s, "GLOBAL_META", "begin_row_index", 0) + 1;
    if (mult <= 0) return fail(s, "row pad multiple <= 0");
    if (rn % (uint64_t)mult == 0) return 0;
    if (!nnz) return fail(s, "row padding of an empty sub-matrix");
    uint64_t add = (rn / mult + 1) * mult - rn, n = nnz + add;
    if ((double)n / (double)nnz >= PADDING_RATE_UP_BOUND) return fail(s, "row padding rate >= %d", PADDING_RATE_UP_BOUND);
    uint64_t *nr = (uint64_t *)malloc(n * 8), *nc = (uint64_t *)malloc(n * 8);
    double *nv = (double *)malloc(n * 8);
    for (uint64_t i = 0; i < nnz; i++) { nr[i] = R->u[i]; nc[i] = C->u[i]; nv[i] = V->f[i]; }
    for (uint64_t i = 0; i < add; i++) { nr[nnz + i] = rn + i; nc[nnz + i] = C->u[nnz - 1]; nv[nnz + i] = 0.0; }
    put_u(s, "GLOBAL_META", "nz_col_indices", 0, nc, n);
    put_f(s, "GLOBAL_META", "nz_vals", 0, nv, n);
    put_u(s, "GLOBAL_META", "nz_row_indices", 0, nr, n);
    return 0;
}

/* modify_{col,vals,row}_*_by_col_pad_parent_blk_to_max_row_size.cc (padding_with_empty_row
 * false): rows [0, row_num), row_num = max(end_row_index, begin + last nonzero's row) - begin
 * + 1 (:40-52); parents = all rows (interval 0, GLOBAL) or fixed row intervals (the parent
 * level's first_row_indices of a fixed row-direction blocking); every non-empty row grows to
 * its parent's longest row, pads repeating the row's last column with value 0 (:54-103). */
static int col_pad_max(or_set *s, uint64_t interval, int with_empty) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t nnz = R->len;
    if (!nnz) return fail(s, "max-row padding of an empty sub-matrix");
    uint64_t b = scalar(s, "GLOBAL_META", "begin_row_index", 0), e = scalar(s, "GLOBAL_META", "end_row_index", 0);
    if (b + R->u[nnz - 1] > e) e = b + R->u[nnz - 1];
    uint64_t row_num = e - b + 1;
    uint64_t *cnt = row_nnz(R->u, nnz, row_num);
    uint64_t *tgt = (uint64_t *)malloc(row_num * 8);
    uint64_t iv = interval ? interval : row_num, after = 0;
    for (uint64_t p0 = 0; p0 < row_num; p0 += iv) {
        uint64_t p1 = p0 + iv < row_num ? p0 + iv : row_num, mx = 0;
        for (uint64_t r = p0; r < p1; r++) if (cnt[r] > mx) mx = cnt[r];
        for (uint64_t r = p0; r < p1; r++) { tgt[r] = (mx && (cnt[r] || with_empty)) ? mx : cnt[r]; after += tgt[r]; }
    }
    if ((double)after / (double)nnz >= PADDING_RATE_UP_BOUND) { /* :95-103 */
        free(cnt); free(tgt);
        return fail(s, "max-row padding rate %.3f >= %d", (double)after / nnz, PADDING_RATE_UP_BOUND);
    }
    uint64_t *nr = (uint64_t *)malloc(after * 8), *nc = (uint64_t *)malloc(after * 8);
    double *nv = (double *)malloc(after * 8);
    uint64_t p = 0, q = 0;
    for (uint64_t r = 0; r < row_num; r++) {
        for (uint64_t k = 0; k < cnt[r]; k++, q++) { nr[p] = R->u[q]; nc[p] = C->u[q]; nv[p] = V->f[q]; p++; }
        /* a pad repeats the last column written so far (the first column before any: :70-72) */
        for (uint64_t k = cnt[r]; k < tgt[r]; k++) { nr[p] = r; nc[p] = p ? nc[p - 1] : C->u[0]; nv[p] = 0.0; p++; }
    }
    free(cnt); free(tgt);
    put_u(s, "GLOBAL_META", "nz_col_indices", 0, nc, after);
    put_f(s, "GLOBAL_META", "nz_vals", 0, nv, after);
    put_u(s, "GLOBAL_META", "nz_row_indices", 0, nr, after);
    return 0;
}

/* ------------------------------------------------------------------ */
/* A5/A7: fixed_interval_row_direction_thread_blocking_operator,        */
/* no-parent branch (operator/...thread_blocking_operator.cc:482-565)   */
/* ------------------------------------------------------------------ */

int or_row_dir_thread_blocking(or_set *s, int rb, int col_pad_size) {
    if (exists(s, "TBLOCK_META", "first_row_indices", 0) || exists(s, "WARP_META", "first_row_indices", 0))
        return fail(s, "oracle restates the no-parent branch only");
    if (col_pad_size > 1 && col_pad(s, col_pad_size)) return -1;
    uint64_t row_num = row_num_of(s);
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    /* get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction.cc:71-97 */
    vu fr = {0};
    int in_bmt = 0, first = 1;
    for (uint64_t i = 0; i < row_num; i++) {
        if (first) { vu_push(&fr, i); first = 0; }
        else in_bmt += 1;
        if (in_bmt == rb) { vu_push(&fr, i); in_bmt = 0; }
    }
    vu_push(&fr, row_num);
    put_u(s, "THREAD_META", "first_row_indices", 0, fr.p, fr.n);
    /* get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction.cc:75-100
     * (row_count / nz_count are `int` in the reference) */
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu fn = {0};
    vu_push(&fn, 0);
    int rc = 0;
    uint64_t nzc = 0;
    for (uint64_t i = 0; i < row_num; i++) {
        rc += 1; nzc += cnt[i];
        if (rc == rb) { vu_push(&fn, nzc); rc = 0; }
    }
    if (rc != rb && rc != 0) vu_push(&fn, nzc);
    free(cnt);
    put_u(s, "THREAD_META", "first_nz_indices", 0, fn.p, fn.n);
    return 0;
}

/* ------------------------------------------------------------------ */
/* A8: fixed_interval_row_direction_tblock_blocking_operator (no pad)   */
/* get_begin_{rows,nzs}_of_BMTBs_after_fixed_blocking_in_row_direction  */
/* ------------------------------------------------------------------ */

static void fixed_row_blocks(or_set *s, int rb, const char *pos) {
    uint64_t row_num = row_num_of(s);
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    vu fr = {0};
    vu_push(&fr, 0);
    uint64_t complete = row_num / rb; /* :74-83 */
    for (uint64_t i = 0; i < complete; i++) vu_push(&fr, (i + 1) * rb);
    if (row_num % rb) vu_push(&fr, row_num);
    put_u(s, pos, "first_row_indices", 0, fr.p, fr.n);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    uint64_t nb = row_num / rb + (row_num % rb ? 1 : 0);
    vu fn = {0};
    vu_push(&fn, 0);
    for (uint64_t i = 0; i < nb; i++) { /* nzs...BMTBs...:70-86 */
        uint64_t c = 0;
        for (uint64_t r = i * rb; r < (i + 1) * rb && r < row_num; r++) c += cnt[r];
        vu_push(&fn, fn.p[fn.n - 1] + c);
    }
    free(cnt);
    put_u(s, pos, "first_nz_indices", 0, fn.p, fn.n);
}

int or_row_dir_tblock_blocking(or_set *s, int rb) {
    if (rb < 1) return fail(s, "rb < 1");
    fixed_row_blocks(s, rb, "TBLOCK_META");
    return 0;
}

/* fixed_interval_row_direction_warp_blocking_operator.cc: without BMTB
 * (get_begin_*_of_BMW_..._without_BMTB.cc) or inside BMTBs
 * (get_begin_*_of_BMW_..._in_BMTB.cc + get_begin_BMWs_of_BMTB_...cc) */
int or_row_dir_warp_blocking(or_set *s, int rb) {
    if (rb < 1) return fail(s, "rb < 1");
    or_array *TR = get(s, "TBLOCK_META", "first_row_indices", 0);
    if (!TR) { fixed_row_blocks(s, rb, "WARP_META"); return 0; }
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu wr = {0}, wn = {0}, tb = {0};
    vu_push(&wn, 0);
    for (uint64_t i = 0; i + 1 < TR->len; i++) {
        uint64_t b = TR->u[i], e = TR->u[i + 1];
        for (uint64_t r0 = b; r0 < e; r0 += rb) {
            vu_push(&wr, r0);
            uint64_t c = 0;
            for (uint64_t r = r0; r < e && r < r0 + rb; r++) c += cnt[r];
            vu_push(&wn, wn.p[wn.n - 1] + c);
        }
    }
    vu_push(&wr, TR->u[TR->len - 1]);
    free(cnt);
    /* get_begin_BMWs_of_BMTB_after_blocking_in_row_direction.cc */
    vu_push(&tb, 0);
    uint64_t cur = 0;
    for (uint64_t i = 0; i + 1 < TR->len; i++) {
        uint64_t e = TR->u[i + 1];
        uint64_t num = 0;
        uint64_t fr = wr.p[cur];
        while (fr < e) {
            num++; cur++;
            if (cur == wr.n) break;
            fr = wr.p[cur];
        }
        vu_push(&tb, tb.p[tb.n - 1] + num);
    }
    put_u(s, "WARP_META", "first_row_indices", 0, wr.p, wr.n);
    put_u(s, "WARP_META", "first_nz_indices", 0, wn.p, wn.n);
    put_u(s, "TBLOCK_META", "first_BMW_indices", 0, tb.p, tb.n);
    return 0;
}

/* ------------------------------------------------------------------ */
/* A9: fixed_interval_nnz_direction_thread_blocking_operator            */
/* (operator/...nnz_direction_thread_blocking_operator.cc:156-245),     */
/* no-parent branch                                                     */
/* ------------------------------------------------------------------ */

int or_nnz_dir_thread_blocking(or_set *s, int nnz_per_bmt, int pad) {
    if (nnz_per_bmt < 1) return fail(s, "nnz_per_BMT < 1");
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t nnz = R->len;
    if (pad && nnz % nnz_per_bmt) { /* modify_*_by_nnz_pad.cc:14-75 */
        uint64_t nn = (nnz / nnz_per_bmt + 1) * nnz_per_bmt;
        if ((double)nn / (double)nnz >= PADDING_RATE_UP_BOUND)
            return fail(s, "nnz padding rate %.3f >= %d", (double)nn / nnz, PADDING_RATE_UP_BOUND);
        or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
        or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
        uint64_t *nc = (uint64_t *)malloc(nn * 8), *nr = (uint64_t *)malloc(nn * 8);
        double *nv = (double *)malloc(nn * 8);
        for (uint64_t i = 0; i < nn; i++) {
            uint64_t k = i < nnz ? i : nnz - 1;
            nc[i] = C->u[k]; nr[i] = R->u[k];
            nv[i] = i < nnz ? V->f[i] : 0.0;
        }
        put_u(s, "GLOBAL_META", "nz_col_indices", 0, nc, nn);
        put_f(s, "GLOBAL_META", "nz_vals", 0, nv, nn);
        put_u(s, "GLOBAL_META", "nz_row_indices", 0, nr, nn);
        R = get(s, "GLOBAL_META", "nz_row_indices", 0);
        nnz = nn;
    }
    uint64_t row_num = row_num_of(s);
    /* get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction.cc */
    vu fr = {0}, fn = {0};
    for (uint64_t i = 0; i < nnz; i += nnz_per_bmt) vu_push(&fr, R->u[i]);
    vu_push(&fr, row_num);
    /* get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction.cc */
    for (uint64_t i = 0; i < nnz; i += nnz_per_bmt) vu_push(&fn, i);
    vu_push(&fn, nnz);
    put_u(s, "THREAD_META", "first_row_indices", 0, fr.p, fr.n);
    put_u(s, "THREAD_META", "first_nz_indices", 0, fn.p, fn.n);
    /* get_BMT_size_of_each_parent.cc (GLOBAL parent): one size when all
     * BMTs are equal, otherwise the item is not created (:118-121) */
    uint64_t size0 = fn.p[1] - fn.p[0];
    int same = 1;
    for (uint64_t i = 0; i + 1 < fn.n; i++)
        if (fn.p[i + 1] - fn.p[i] != size0) { same = 0; break; }
    if (same) put_scalar(s, "GLOBAL_META", "BMT_size_of_each_blk", 0, size0);
    return 0;
}

/* ------------------------------------------------------------------ */
/* nnz-direction BMTB / BMW blocking and BMTs inside them               */
/* fixed_interval_nnz_direction_{tblock,warp,thread}_blocking_operator  */
/* ------------------------------------------------------------------ */

/* modify_{col,val,row}_*_by_nnz_pad.cc:14-75: pad the COO to a multiple of k with copies
 * of the last entry's row / column and value 0 */
static int nnz_pad_to(or_set *s, uint64_t k) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t nnz = R->len;
    if (nnz % k == 0) return 0;
    uint64_t nn = (nnz / k + 1) * k;
    if ((double)nn / (double)nnz >= PADDING_RATE_UP_BOUND)
        return fail(s, "nnz padding rate %.3f >= %d", (double)nn / nnz, PADDING_RATE_UP_BOUND);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t *nc = (uint64_t *)malloc(nn * 8), *nr = (uint64_t *)malloc(nn * 8);
    double *nv = (double *)malloc(nn * 8);
    for (uint64_t i = 0; i < nn; i++) {
        uint64_t q = i < nnz ? i : nnz - 1;
        nc[i] = C->u[q]; nr[i] = R->u[q];
        nv[i] = i < nnz ? V->f[i] : 0.0;
    }
    put_u(s, "GLOBAL_META", "nz_col_indices", 0, nc, nn);
    put_f(s, "GLOBAL_META", "nz_vals", 0, nv, nn);
    put_u(s, "GLOBAL_META", "nz_row_indices", 0, nr, nn);
    return 0;
}

/* get_begin_{rows,nzs}_of_<unit>_after_fixed_blocking_in_nnz_direction.cc: a unit every k
 * nonzeros, its row = the row of that nonzero, the row array closed by the row count */
static void nnz_units(or_set *s, const char *pos, uint64_t k) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t nnz = R->len, row_num = row_num_of(s);
    vu fr = {0}, fn = {0};
    for (uint64_t i = 0; i < nnz; i += k) { vu_push(&fr, R->u[i]); vu_push(&fn, i); }
    vu_push(&fr, row_num);
    vu_push(&fn, nnz);
    put_u(s, pos, "first_row_indices", 0, fr.p, fr.n);
    put_u(s, pos, "first_nz_indices", 0, fn.p, fn.n);
}

/* *_relative_to_{BMTB,BMW}.cc:25-45: the parent id moves on by one (an `if`) when a unit
 * start reaches the next parent's first nonzero */
static void nnz_units_relative(or_set *s, const char *pos, const char *parent, const char *suffix, uint64_t k,
                               int rows, int nzs) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *PN = get(s, parent, "first_nz_indices", 0), *PR = get(s, parent, "first_row_indices", 0);
    vu rr = {0}, rn = {0};
    uint64_t pid = 0;
    for (uint64_t i = 0; i < R->len; i += k) {
        if (i >= PN->u[pid + 1]) pid++;
        vu_push(&rr, R->u[i] - PR->u[pid]);
        vu_push(&rn, i - PN->u[pid]);
    }
    char nr_[64], nn_[64];
    snprintf(nr_, sizeof nr_, "first_row_indices_relative_to_%s", suffix);
    snprintf(nn_, sizeof nn_, "first_nz_indices_relative_to_%s", suffix);
    if (rows) put_u(s, pos, nr_, 0, rr.p, rr.n); else free(rr.p);
    if (nzs) put_u(s, pos, nn_, 0, rn.p, rn.n); else free(rn.p);
}

/* get_begin_BMWs_of_BMTB_after_blocking.cc / get_begin_BMTs_of_specific_parent_after_blocking.cc:
 * the first child of every parent */
static int children_of(or_set *s, const char *child, const char *parent, const char *name) {
    or_array *CN = get(s, child, "first_nz_indices", 0), *PN = get(s, parent, "first_nz_indices", 0);
    vu out = {0};
    vu_push(&out, 0);
    uint64_t cur = 0;
    for (uint64_t p = 0; p + 1 < PN->len; p++) {
        if (CN->u[cur] != PN->u[p]) { free(out.p); return fail(s, "a parent does not start on a child"); }
        uint64_t num = 0;
        while (CN->u[cur] < PN->u[p + 1]) { num++; cur++; }
        vu_push(&out, out.p[out.n - 1] + num);
    }
    put_u(s, parent, name, 0, out.p, out.n);
    return 0;
}

/* one size when every unit of the level has the same number of nonzeros (GLOBAL parent) */
static int same_size(or_set *s, const char *pos, uint64_t *size) {
    or_array *FN = get(s, pos, "first_nz_indices", 0);
    *size = FN->u[1] - FN->u[0];
    for (uint64_t i = 0; i + 1 < FN->len; i++)
        if (FN->u[i + 1] - FN->u[i] != *size) return 0;
    return 1;
}

static int has_level(or_set *s, const char *pos) {
    size_t n = strlen(pos);
    for (int i = 0; i < s->n; i++)
        if (!strncmp(s->a[i].key, pos, n)) return 1;
    return 0;
}

int or_nnz_dir_tblock_blocking(or_set *s, uint64_t k, int pad) {
    /* fixed_interval_nnz_direction_tblock_blocking_operator.cc:50-135 */
    if (has_level(s, "THREAD_META") || has_level(s, "WARP_META") || has_level(s, "TBLOCK_META"))
        return fail(s, "nnz-direction tblock blocking after other blocking (:63-70)");
    if (pad && nnz_pad_to(s, k)) return -1;
    nnz_units(s, "TBLOCK_META", k);
    uint64_t sz;
    if (pad) {
        if (!same_size(s, "TBLOCK_META", &sz)) return fail(s, "BMTB sizes differ (get_BMTB_size.cc:81-85)");
        put_scalar(s, "GLOBAL_META", "BMTB_size_of_each_blk", 0, sz);
    }
    return 0;
}

int or_nnz_dir_warp_blocking(or_set *s, uint64_t k, int rrel, int nrel, int pad) {
    /* fixed_interval_nnz_direction_warp_blocking_operator.cc:87-200 */
    int bmtb = exists(s, "TBLOCK_META", "first_row_indices", 0);
    if (has_level(s, "THREAD_META") || has_level(s, "WARP_META")) return fail(s, "warp level exists (:95-99)");
    if ((rrel || nrel) && !bmtb) return fail(s, "relative BMW indices without a BMTB (:102-105)");
    if (pad && bmtb) return fail(s, "nnz padding inside a BMTB (:106-109)");
    if (bmtb) {
        or_array *PN = get(s, "TBLOCK_META", "first_nz_indices", 0);
        uint64_t bsz = PN->u[1] - PN->u[0];
        if (bsz % k) return fail(s, "nnz_per_BMTB %% nnz_per_BMW != 0 (:60-70)");
    }
    if (pad && nnz_pad_to(s, k)) return -1;
    nnz_units(s, "WARP_META", k);
    if (rrel || nrel) nnz_units_relative(s, "WARP_META", "TBLOCK_META", "BMTB", k, rrel, nrel);
    if (bmtb && children_of(s, "WARP_META", "TBLOCK_META", "first_BMW_indices")) return -1;
    uint64_t sz;
    if (same_size(s, "WARP_META", &sz)) put_scalar(s, "GLOBAL_META", "BMW_size_of_each_blk", 0, sz);
    return 0;
}

/* BMTs inside an nnz-direction parent (fixed_interval_nnz_direction_thread_blocking_operator.cc:156-245) */
int or_nnz_dir_thread_in_parent(or_set *s, uint64_t k, int rrel, int nrel) {
    int bmw = exists(s, "WARP_META", "first_row_indices", 0), bmtb = exists(s, "TBLOCK_META", "first_row_indices", 0);
    if (!bmw && !bmtb) return fail(s, "no parent level");
    const char *par = bmw ? "WARP_META" : "TBLOCK_META";
    or_array *PN = get(s, par, "first_nz_indices", 0);
    if ((PN->u[1] - PN->u[0]) % k) return fail(s, "parent size %% nnz_per_BMT != 0 (:66-90)");
    nnz_units(s, "THREAD_META", k);
    if (rrel || nrel) nnz_units_relative(s, "THREAD_META", par, bmw ? "BMW" : "BMTB", k, rrel, nrel);
    if (children_of(s, "THREAD_META", par, "first_BMT_indices")) return -1;
    uint64_t sz;
    if (same_size(s, "THREAD_META", &sz)) put_scalar(s, "GLOBAL_META", "BMT_size_of_each_blk", 0, sz);
    return 0;
}

/* ------------------------------------------------------------------ */
/* thread_bit_map_operator.cc:60-101 and its transforms                 */
/* ------------------------------------------------------------------ */

int or_thread_bit_map_operator(or_set *s, int pos_is_warp, int size) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *FN = get(s, "THREAD_META", "first_nz_indices", 0);
    if (!R || !FN) return fail(s, "missing THREAD first_nz_indices");
    uint64_t nnz = R->len, nb = FN->len - 1;
    if (FN->u[nb] != nnz) return fail(s, "bitmap length mismatch (thread_bit_map.cc:43)");
    /* thread_bit_map.cc:27-41 */
    unsigned char *bit = (unsigned char *)malloc(nnz);
    bit[0] = 1;
    for (uint64_t j = 1; j < nnz; j++) bit[j] = R->u[j] != R->u[j - 1];
    /* thread_bit_map.cc:45-71: with a WARP/TBLOCK parent, the head of
     * every size-th BMT is forced to 1.  thread_size is read from the
     * GLOBAL BMT_size_of_each_blk; the reference divides by zero without
     * it, and writes one element past the end when nb % size == 0 -- that
     * write never reaches an output array, so it is skipped here. */
    if (pos_is_warp) {
        if (!exists(s, "GLOBAL_META", "BMT_size_of_each_blk", 0)) {
            free(bit);
            return fail(s, "GLOBAL BMT_size_of_each_blk missing: reference divides by zero (thread_bit_map.cc:56)");
        }
        uint64_t ts = FN->u[1] - FN->u[0];
        for (uint64_t i = 0; i < nnz / ts + 1; i += (uint64_t)size)
            if (i * ts < nnz) bit[i * ts] = 1;
    }
    /* thread_bit_map.cc:74-90: LSB = first nz of the BMT */
    uint64_t *tbm = (uint64_t *)malloc(nb * 8);
    for (uint64_t i = 0; i < nb; i++) {
        uint64_t m = 0;
        for (uint64_t j = FN->u[i + 1]; j-- > FN->u[i];) m = (m << 1) | bit[j];
        tbm[i] = m;
    }
    free(bit);
    put_u(s, "THREAD_META", "thread_bit_map", 0, tbm, nb);

    /* segment_empty_flag.cc:14-75 */
    unsigned char *flag = (unsigned char *)calloc(nb ? nb : 1, 1);
    for (uint64_t j = 0; j < nb; j++) {
        for (uint64_t i = FN->u[j] + 1; i < FN->u[j + 1]; i++)
            if (R->u[i] - R->u[i - 1] > 1) { flag[j] = 1; break; }
    }
    vu sef = {0};
    for (uint64_t i = 0; i < nb; i += (uint64_t)size) {
        uint64_t k = (i + size - 1) > (nb - 1) ? (nb - 1) : (i + size - 1);
        uint64_t cur = 0;
        for (uint64_t j = k + 1; j-- > i;) cur = (cur << 1) | flag[j];
        vu_push(&sef, cur);
    }
    free(flag);
    put_u(s, "THREAD_META", "segment_empty_flag", 0, sef.p, sef.n);

    /* segment_empty_row_indices.cc */
    vu seri = {0};
    for (uint64_t j = 0; j < nb; j++) {
        uint64_t first_row = R->u[FN->u[j]];
        vu_push(&seri, 0);
        for (uint64_t i = FN->u[j] + 1; i < FN->u[j + 1]; i++)
            if (R->u[i] != R->u[i - 1]) vu_push(&seri, R->u[i] - first_row);
    }
    put_u(s, "THREAD_META", "segment_empty_row_indices", 0, seri.p, seri.n);

    /* segment_offset.cc (parent_flag=false as called from
     * thread_bit_map_operator.cc:81): the count pending after the last
     * non-empty bitmap is never written back (reference behaviour). */
    uint64_t *so = (uint64_t *)calloc(nb ? nb : 1, 8);
    uint64_t count = 0, prev = 0;
    for (uint64_t j = 1; j < nb; j++) {
        if (tbm[j] == 0) count++;
        else { so[prev] = count; count = 0; prev = j; }
    }
    put_u(s, "THREAD_META", "segment_offset", 0, so, nb);

    /* segment_ptr.cc: running count of row segments, one entry per BMT,
     * the last BMT's segments are not counted */
    vu sp = {0};
    vu_push(&sp, 0);
    uint64_t c = 0;
    for (uint64_t j = 0; j + 2 < FN->len; j++) {
        c += 1;
        for (uint64_t i = FN->u[j] + 1; i < FN->u[j + 1]; i++)
            if (R->u[i] != R->u[i - 1]) c += 1;
        vu_push(&sp, c);
    }
    put_u(s, "THREAD_META", "segment_ptr", 0, sp.p, sp.n);
    return 0;
}

/* warp_segment_reduce_operator.cc:74-111 with merge_num = VECTOR_WIDTH:
 * get_begin_rows_after_merge_thread.cc, get_begin_nzs_after_merge_thread.cc,
 * get_begin_BMTs_after_merge_thread.cc */
int or_warp_segment_operator(or_set *s, int vw) {
    or_array *TR = get(s, "THREAD_META", "first_row_indices", 0);
    or_array *TN = get(s, "THREAD_META", "first_nz_indices", 0);
    if (!TR || !TN || vw < 1) return fail(s, "warp_segment: missing THREAD arrays");
    vu wr = {0}, wn = {0}, wb = {0};
    for (uint64_t j = 0; j + 1 < TR->len; j += vw) vu_push(&wr, TR->u[j]);
    vu_push(&wr, TR->u[TR->len - 1]);
    for (uint64_t j = 0; j + 1 < TN->len; j += vw) vu_push(&wn, TN->u[j]);
    vu_push(&wn, TN->u[TN->len - 1]);
    for (uint64_t j = 0; j + 1 < TN->len; j += vw) vu_push(&wb, j);
    vu_push(&wb, TN->len - 1);
    put_u(s, "WARP_META", "first_row_indices", 0, wr.p, wr.n);
    put_u(s, "WARP_META", "first_nz_indices", 0, wn.p, wn.n);
    put_u(s, "WARP_META", "first_BMT_indices", 0, wb.p, wb.n);
    return 0;
}

/* ------------------------------------------------------------------ */
/* A10: fixed_interval_col_direction_thread_blocking_operator, no-parent */
/* branch (operator/...col_direction_thread_blocking_operator.cc:285-509) */
/* ------------------------------------------------------------------ */

int or_col_dir_thread_blocking(or_set *s, int col_size, int pad) {
    if (col_size < 1) return fail(s, "fixed_col_block_size < 1");
    if (exists(s, "TBLOCK_META", "first_row_indices", 0) || exists(s, "WARP_META", "first_row_indices", 0))
        return fail(s, "oracle restates the no-parent branch only");
    /* :313-326 -> modify_{col,val,row}_by_col_pad_in_sub_matrix (A6); the
     * padding-rate rule is data_transform_common.cc:644-690 */
    if (pad && col_pad(s, col_size)) return -1;
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t nnz = R->len, row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, nnz, row_num);
    /* get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction.cc:136-160 */
    vu fr = {0};
    for (uint64_t i = 0; i < row_num; i++) {
        uint64_t k = cnt[i] / col_size;
        if (cnt[i] % col_size != 0) k = k + 1;
        for (uint64_t j = 0; j < k; j++) vu_push(&fr, i);
    }
    /* get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction.cc:124-150 */
    vu fn = {0};
    vu_push(&fn, 0);
    for (uint64_t i = 0; i < row_num; i++) {
        int64_t remain = (int64_t)cnt[i];
        while (remain > 0) {
            if (remain < col_size) { vu_push(&fn, fn.p[fn.n - 1] + remain); remain = 0; }
            else { vu_push(&fn, fn.p[fn.n - 1] + col_size); remain -= col_size; }
        }
    }
    free(cnt);
    put_u(s, "THREAD_META", "first_row_indices_without_ending", 0, fr.p, fr.n);
    put_u(s, "THREAD_META", "first_nz_indices", 0, fn.p, fn.n);
    /* :477-482 get_BMT_size_of_each_parent (GLOBAL): one size when all equal */
    if (pad) {
        uint64_t size0 = fn.p[1] - fn.p[0];
        int same = 1;
        for (uint64_t i = 0; i + 1 < fn.n; i++)
            if (fn.p[i + 1] - fn.p[i] != size0) { same = 0; break; }
        if (same) put_scalar(s, "GLOBAL_META", "BMT_size_of_each_blk", 0, size0);
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* col-direction BMWs / BMTBs and BMTs inside row-direction parents     */
/* fixed_interval_col_direction_{tblock,warp,thread}_blocking_operator  */
/* ------------------------------------------------------------------ */

/* get_begin_{rows,nzs}_of_{BMW,BMTB}_after_fixed_blocking_in_col_direction.cc:75-105: a unit
 * per chunk of c nonzeros of one row; rows without ending, nz starts closed by nnz */
static void col_units(or_set *s, const char *pos, uint64_t c) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu fr = {0}, fn = {0};
    vu_push(&fn, 0);
    for (uint64_t i = 0; i < row_num; i++) {
        int64_t remain = (int64_t)cnt[i];
        while (remain > 0) {
            uint64_t t = remain < (int64_t)c ? (uint64_t)remain : c;
            vu_push(&fr, i);
            vu_push(&fn, fn.p[fn.n - 1] + t);
            remain -= (int64_t)t;
        }
    }
    free(cnt);
    put_u(s, pos, "first_row_indices_without_ending", 0, fr.p, fr.n);
    put_u(s, pos, "first_nz_indices", 0, fn.p, fn.n);
}

/* get_begin_rows_of_<unit>_after_fixed_blocking_in_col_direction_relative_to_<P>.cc:85-120 and
 * get_begin_nzs_of_..._relative_to_{BMTB,parents}.cc:100-170: per parent block, the chunks of
 * its rows; rows minus the parent's first row, nz starts from 0 (a 0 pushed per parent, the
 * parent's closing offset popped) */
static void col_units_relative(or_set *s, const char *pos, const char *parent, const char *tag, uint64_t c, int rows,
                               int nzs) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0), *PR = get(s, parent, "first_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu rr = {0}, rn = {0};
    for (uint64_t p = 0; p + 1 < PR->len; p++) {
        vu off = {0};
        vu_push(&off, 0);
        for (uint64_t r = PR->u[p]; r < PR->u[p + 1]; r++) {
            int64_t remain = (int64_t)(r < row_num ? cnt[r] : 0);
            while (remain > 0) {
                uint64_t t = remain < (int64_t)c ? (uint64_t)remain : c;
                vu_push(&rr, r - PR->u[p]);
                vu_push(&off, off.p[off.n - 1] + t);
                remain -= (int64_t)t;
            }
        }
        for (uint64_t k = 0; k + 1 < off.n; k++) vu_push(&rn, off.p[k]); /* pop_back of the last */
        free(off.p);
    }
    free(cnt);
    char k1[64], k2[64];
    snprintf(k1, sizeof k1, "first_row_indices_relative_to_%s", tag);
    snprintf(k2, sizeof k2, "first_nz_indices_relative_to_%s", tag);
    if (rows) put_u(s, pos, k1, 0, rr.p, rr.n); else free(rr.p);
    if (nzs) put_u(s, pos, k2, 0, rn.p, rn.n); else free(rn.p);
}

/* get_BMT_size_of_each_parent.cc (parent level, row_direction_blocking false): the BMT size of
 * every parent block (0 for a parent without BMTs), no item when one parent mixes sizes */
static void unit_sizes_per_parent(or_set *s, const char *child, const char *parent, const char *name) {
    or_array *CN = get(s, child, "first_nz_indices", 0), *PN = get(s, parent, "first_nz_indices", 0);
    vu out = {0};
    uint64_t cur = 0;
    for (uint64_t p = 0; p + 1 < PN->len; p++) {
        uint64_t sz = 0;
        int seen = 0;
        while (cur + 1 < CN->len && CN->u[cur] < PN->u[p + 1]) {
            uint64_t b = CN->u[cur + 1] - CN->u[cur];
            if (!seen) { sz = b; seen = 1; }
            else if (b != sz) { free(out.p); return; }
            cur++;
        }
        vu_push(&out, sz);
    }
    put_u(s, parent, name, 0, out.p, out.n);
}

int or_col_dir_tblock_blocking(or_set *s, uint64_t c, int pad) {
    /* fixed_interval_col_direction_tblock_blocking_operator.cc:80-201 */
    if (c < 1) return fail(s, "fixed_col_block_size < 1");
    if (has_level(s, "THREAD_META") || has_level(s, "WARP_META") || has_level(s, "TBLOCK_META"))
        return fail(s, "col-direction tblock blocking after other blocking (:94-99)");
    if (pad && col_pad(s, (int)c)) return -1;
    col_units(s, "TBLOCK_META", c);
    uint64_t sz;
    if (pad) {
        if (!same_size(s, "TBLOCK_META", &sz)) return fail(s, "BMTB sizes differ (get_BMTB_size.cc:81-85)");
        put_scalar(s, "GLOBAL_META", "BMTB_size_of_each_blk", 0, sz);
    }
    return 0;
}

int or_col_dir_warp_blocking(or_set *s, uint64_t c, int rrel, int nrel) {
    /* fixed_interval_col_direction_warp_blocking_operator.cc:102-372 (no padding) */
    int bmtb = exists(s, "TBLOCK_META", "first_row_indices", 0);
    if (c < 1) return fail(s, "fixed_col_block_size < 1");
    if (has_level(s, "THREAD_META") || has_level(s, "WARP_META")) return fail(s, "warp level exists (:118-124)");
    if ((rrel || nrel) && !bmtb) return fail(s, "relative BMW indices without a BMTB (:126-134)");
    col_units(s, "WARP_META", c);
    if (rrel || nrel) col_units_relative(s, "WARP_META", "TBLOCK_META", "BMTB", c, rrel, nrel);
    if (bmtb && children_of(s, "WARP_META", "TBLOCK_META", "first_BMW_indices")) return -1;
    return 0;
}

/* col-direction BMTs inside the nearest row-direction parent (a BMW, else a BMTB), relative
 * indices to it, the parent's first BMT per block; pad = rows padded to a multiple of c first
 * (the reference pads, drops the parent level and re-runs its operator on the padded COO --
 * the caller runs the parent blocking after or_col_pad_rows) and the BMT sizes */
int or_col_dir_thread_in_parent(or_set *s, uint64_t c, int rrel, int nrel, int pad) {
    int bmw = exists(s, "WARP_META", "first_row_indices", 0), bmtb = exists(s, "TBLOCK_META", "first_row_indices", 0);
    if (!bmw && !bmtb) return fail(s, "no parent level");
    if (c < 1) return fail(s, "fixed_col_block_size < 1");
    const char *par = bmw ? "WARP_META" : "TBLOCK_META";
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu fr = {0}, fn = {0};
    vu_push(&fn, 0);
    for (uint64_t i = 0; i < row_num; i++) { /* get_begin_{rows,nzs}_of_BMT_..._in_col_direction.cc */
        int64_t remain = (int64_t)cnt[i];
        while (remain > 0) {
            uint64_t t = remain < (int64_t)c ? (uint64_t)remain : c;
            vu_push(&fr, i);
            vu_push(&fn, fn.p[fn.n - 1] + t);
            remain -= (int64_t)t;
        }
    }
    free(cnt);
    put_u(s, "THREAD_META", "first_row_indices_without_ending", 0, fr.p, fr.n);
    put_u(s, "THREAD_META", "first_nz_indices", 0, fn.p, fn.n);
    if (rrel || nrel) col_units_relative(s, "THREAD_META", par, bmw ? "BMW" : "BMTB", c, rrel, nrel);
    if (bmtb && children_of(s, "THREAD_META", "TBLOCK_META", "first_BMT_indices")) return -1;
    if (pad && bmtb) unit_sizes_per_parent(s, "THREAD_META", "TBLOCK_META", "BMT_size_of_each_blk");
    if (bmw && children_of(s, "THREAD_META", "WARP_META", "first_BMT_indices")) return -1;
    if (pad && bmw) unit_sizes_per_parent(s, "THREAD_META", "WARP_META", "BMT_size_of_each_blk");
    uint64_t sz;
    if (pad && same_size(s, "THREAD_META", &sz)) put_scalar(s, "GLOBAL_META", "BMT_size_of_each_blk", 0, sz);
    return 0;
}

/* warp_bit_map_operator.cc:69-109 (pos_is_warp = 1, merge = VECTOR_WIDTH) and
 * tblock_thread_bit_map_operator.cc:62-109 (pos_is_warp = 0, merge = block_size):
 * get_begin_{rows,nzs}_after_merge_thread.cc, the relative variants
 * get_begin_{rows,nzs}_relative_to_parent_after_merge_thread.cc,
 * get_begin_BMTs_after_merge_thread.cc, parent_bit_map_of_thread.cc and, for
 * the TBLOCK parent, segment_offset.cc (parent_flag = true: the POS_TYPE
 * argument TBLOCK_META = -98 converts to true). */
int or_parent_bit_map_operator(or_set *s, int pos_is_warp, int merge, int rel_nz, int rel_row) {
    const char *pos = pos_is_warp ? "WARP_META" : "TBLOCK_META";
    or_array *TR = get(s, "THREAD_META", "first_row_indices_without_ending", 0);
    or_array *TN = get(s, "THREAD_META", "first_nz_indices", 0);
    if (!TR || !TN || merge < 1) return fail(s, "bit-map operator: needs col-direction BMTs");
    vu pr = {0}, pn = {0}, pb = {0};
    for (uint64_t j = 0; j + 1 < TR->len; j += merge) vu_push(&pr, TR->u[j]);
    vu_push(&pr, TR->u[TR->len - 1]);
    for (uint64_t j = 0; j + 1 < TN->len; j += merge) vu_push(&pn, TN->u[j]);
    vu_push(&pn, TN->u[TN->len - 1]);
    put_u(s, pos, "first_row_indices", 0, pr.p, pr.n);
    put_u(s, pos, "first_nz_indices", 0, pn.p, pn.n);
    TR = get(s, "THREAD_META", "first_row_indices_without_ending", 0);
    TN = get(s, "THREAD_META", "first_nz_indices", 0);
    if (rel_row) { /* loop bound len-1: the last BMT gets no entry */
        vu rr = {0};
        for (uint64_t j = 0; j + 1 < TR->len; j += merge)
            for (uint64_t i = j; i < j + merge && i + 1 < TR->len; i++) vu_push(&rr, TR->u[i] - TR->u[j]);
        put_u(s, pos, pos_is_warp ? "first_row_indices_relative_to_BMW" : "first_row_indices_relative_to_BMTB", 0,
              rr.p, rr.n);
        TR = get(s, "THREAD_META", "first_row_indices_without_ending", 0);
        TN = get(s, "THREAD_META", "first_nz_indices", 0);
    }
    if (rel_nz) {
        vu rn = {0};
        for (uint64_t j = 0; j + 1 < TN->len; j += merge)
            for (uint64_t i = j; i < j + merge && i + 1 < TN->len; i++) vu_push(&rn, TN->u[i] - TN->u[j]);
        put_u(s, "THREAD_META", pos_is_warp ? "first_nz_indices_relative_to_BMW" : "first_nz_indices_relative_to_BMTB",
              0, rn.p, rn.n);
        TR = get(s, "THREAD_META", "first_row_indices_without_ending", 0);
        TN = get(s, "THREAD_META", "first_nz_indices", 0);
    }
    for (uint64_t j = 0; j + 1 < TN->len; j += merge) vu_push(&pb, j);
    vu_push(&pb, TN->len - 1);
    put_u(s, pos, "first_BMT_indices", 0, pb.p, pb.n);
    TR = get(s, "THREAD_META", "first_row_indices_without_ending", 0);
    /* parent_bit_map_of_thread.cc */
    uint64_t n = TR->len;
    unsigned char *bit = (unsigned char *)calloc(n ? n : 1, 1);
    bit[0] = 1;
    for (uint64_t j = 1; j < n; j++) bit[j] = TR->u[j] != TR->u[j - 1];
    if (pos_is_warp) {
        for (uint64_t i = 0; i < n; i += merge) bit[i] = 1;
        vu bm = {0};
        for (uint64_t i = 0; i < n; i += merge) {
            uint64_t k = (i + merge - 1) > (n - 1) ? (n - 1) : (i + merge - 1);
            uint64_t map = 0;
            for (uint64_t j = k;; j--) {
                map = (map << 1) | bit[j];
                if (j == i) break;
            }
            vu_push(&bm, map);
        }
        put_u(s, "WARP_META", "bit_map_of_thread", 0, bm.p, bm.n);
    } else {
        or_array *FB = get(s, "TBLOCK_META", "first_BMT_indices", 0);
        for (uint64_t i = 0; i < FB->len; i++)
            if (FB->u[i] < n) bit[FB->u[i]] = 1; /* the ending (= n) lands past the end in the reference */
        uint64_t *bm = (uint64_t *)malloc(n * 8);
        for (uint64_t i = 0; i < n; i++) bm[i] = bit[i];
        put_u(s, "THREAD_META", "bit_map_of_thread", 0, bm, n);
        /* segment_offset.cc with parent_flag = true, size = block_size */
        uint64_t *so = (uint64_t *)calloc(n ? n : 1, 8);
        uint64_t count = 0, prev = 0;
        for (uint64_t j = 1; j < n; j++) {
            if (bit[j] == 0 && (j % (uint64_t)merge != 0)) count++;
            else { so[prev] = count; count = 0; prev = j; }
        }
        put_u(s, "THREAD_META", "segment_offset", 0, so, n);
    }
    free(bit);
    return 0;
}

/* A11: balanced_interval_row_direction_warp_blocking_operator, no-parent
 * branch; split points data_transform_common.cc:934-989 */
int or_balanced_row_dir_warp_blocking(or_set *s, uint64_t per) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu br = {0}, bn = {0};
    vu_push(&br, 0);
    uint64_t nzc = 0;
    for (uint64_t i = 0; i < row_num; i++) {
        nzc += cnt[i];
        if (nzc >= per) { vu_push(&br, i + 1); nzc = 0; }
    }
    if (br.p[br.n - 1] < row_num) {
        if (nzc == 0) { free(cnt); free(br.p); return fail(s, "trailing empty rows after last cut (data_transform_common.cc:984)"); }
        vu_push(&br, row_num);
    }
    vu_push(&bn, 0);
    uint32_t c32 = 0, tot32 = 0; /* `unsigned int` counters, :938-939 */
    for (uint64_t i = 0; i < row_num; i++) {
        c32 += (uint32_t)cnt[i]; tot32 += (uint32_t)cnt[i];
        if (c32 >= per) { vu_push(&bn, tot32); c32 = 0; }
    }
    if (c32 != 0) vu_push(&bn, tot32);
    free(cnt);
    put_u(s, "WARP_META", "first_row_indices", 0, br.p, br.n);
    put_u(s, "WARP_META", "first_nz_indices", 0, bn.p, bn.n);
    return 0;
}

/* A11 at TBLOCK level: balanced_interval_row_direction_tblock_blocking_operator.cc:89-120
 * (get_begin_{rows,nzs}_of_BMTB_after_nnz_blocking_in_row_direction.cc: the same
 * split points as the BMW version, written to TBLOCK_META) */
static int balanced_split(or_set *s, uint64_t per, const char *pos) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu br = {0}, bn = {0};
    vu_push(&br, 0);
    uint64_t nzc = 0;
    for (uint64_t i = 0; i < row_num; i++) { /* data_transform_common.cc:960-989 */
        nzc += cnt[i];
        if (nzc >= per) { vu_push(&br, i + 1); nzc = 0; }
    }
    if (br.p[br.n - 1] < row_num) {
        if (nzc == 0) { free(cnt); free(br.p); return fail(s, "trailing empty rows after last cut (data_transform_common.cc:984)"); }
        vu_push(&br, row_num);
    }
    vu_push(&bn, 0);
    uint32_t c32 = 0, tot32 = 0; /* data_transform_common.cc:934-957, `unsigned int` counters */
    for (uint64_t i = 0; i < row_num; i++) {
        c32 += (uint32_t)cnt[i]; tot32 += (uint32_t)cnt[i];
        if (c32 >= per) { vu_push(&bn, tot32); c32 = 0; }
    }
    if (c32 != 0) vu_push(&bn, tot32);
    free(cnt);
    put_u(s, pos, "first_row_indices", 0, br.p, br.n);
    put_u(s, pos, "first_nz_indices", 0, bn.p, bn.n);
    return 0;
}

int or_balanced_row_dir_tblock_blocking(or_set *s, uint64_t per) { return balanced_split(s, per, "TBLOCK_META"); }

/* A11 at WARP level inside BMTBs: balanced_interval_row_direction_warp_blocking_operator.cc:165-207
 * with data_transform_common.cc:794-901: per BMTB a new BMW after the row whose running count
 * reaches per, never at the BMTB's last row; absolute arrays end with row_num / the last BMTB
 * nz, relative ones restart at 0 and have no ending; first_BMW_indices = BMWs before each BMTB */
static int or_balanced_in_parent(or_set *s, uint64_t per, int rel, const char *child, const char *parent,
                                 const char *rel_suffix, const char *first_child) {
    if (!per) return fail(s, "nnz_per_interval > 0");
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    if (!R->len) return fail(s, "balanced BMWs of an empty sub-matrix");
    uint64_t b = scalar(s, "GLOBAL_META", "begin_row_index", 0), e = scalar(s, "GLOBAL_META", "end_row_index", 0);
    if (b + R->u[R->len - 1] > e) e = b + R->u[R->len - 1];
    uint64_t row_num = e - b + 1;
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    or_array *PR = get(s, parent, "first_row_indices", 0), *PN = get(s, parent, "first_nz_indices", 0);
    vu rows = {0}, rrel = {0}, nzs = {0}, nrel = {0}, fb = {0};
    for (uint64_t j = 0; j + 1 < PR->len; j++) {
        vu_push(&fb, rows.n);
        vu_push(&rows, PR->u[j]); vu_push(&rrel, 0); vu_push(&nzs, PN->u[j]); vu_push(&nrel, 0);
        uint64_t run = 0, in_blk = 0;
        for (uint64_t i = PR->u[j]; i < PR->u[j + 1]; i++) {
            run += cnt[i]; in_blk += cnt[i];
            if (run >= per && i != PR->u[j + 1] - 1) {
                vu_push(&rows, i + 1); vu_push(&rrel, i + 1 - PR->u[j]);
                vu_push(&nzs, PN->u[j] + in_blk); vu_push(&nrel, in_blk);
                run = 0;
            }
        }
    }
    vu_push(&fb, rows.n);
    vu_push(&rows, row_num);
    vu_push(&nzs, PN->u[PN->len - 1]);
    free(cnt);
    char nm[96];
    put_u(s, child, "first_row_indices", 0, rows.p, rows.n);
    put_u(s, child, "first_nz_indices", 0, nzs.p, nzs.n);
    if (rel) {
        snprintf(nm, sizeof nm, "first_row_indices_relative_to_%s", rel_suffix);
        put_u(s, child, nm, 0, rrel.p, rrel.n);
        snprintf(nm, sizeof nm, "first_nz_indices_relative_to_%s", rel_suffix);
        put_u(s, child, nm, 0, nrel.p, nrel.n);
    } else { free(rrel.p); free(nrel.p); }
    put_u(s, parent, first_child, 0, fb.p, fb.n);
    return 0;
}
static int or_balanced_bmw_in_bmtb(or_set *s, uint64_t per, int rel) {
    return or_balanced_in_parent(s, per, rel, "WARP_META", "TBLOCK_META", "BMTB", "first_BMW_indices");
}

/* A11 at THREAD level, no parent: balanced_interval_row_direction_thread_blocking_operator.cc
 * (get_begin_{rows,nzs}_of_BMT_after_nnz_blocking_in_row_direction.cc:60-88) */
int or_balanced_row_dir_thread_blocking(or_set *s, uint64_t per) { return balanced_split(s, per, "THREAD_META"); }

/* A11 merge path: get_begin_rows_of_level_after_merge_path.cc:43-98 and
 * get_begin_nzs_of_level_after_merge_path.cc:43-102, written literally (the
 * quadratic first-match search over total_path for every level start). */
int or_merge_path(or_set *s, const char *pos, uint64_t work_size) {
    if (work_size == 0) return fail(s, "work_size > 0");
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu total_path = {0}, path_row = {0}, lr = {0}, ln = {0};
    uint64_t count = 0;
    int flag = 1;
    for (uint64_t i = 0; i < row_num; i++) { /* :64-79 */
        if (cnt[i] != 0) {
            count += 1;
            if (flag) { flag = 0; count -= 1; }
            count += cnt[i];
            vu_push(&total_path, count);
            vu_push(&path_row, i);
        }
    }
    free(cnt);
    for (uint64_t i = 0; i < count; i += work_size) { /* :84-94 */
        for (uint64_t j = 0; j < total_path.n; j++) {
            if (total_path.p[j] > i) {
                vu_push(&lr, path_row.p[j]);
                vu_push(&ln, i - j);
                break;
            }
        }
    }
    vu_push(&ln, R->len); /* nzs :95 */
    free(total_path.p);
    free(path_row.p);
    if (lr.n == 0) { free(ln.p); return fail(s, "merge path over a sub-matrix without nonzeros"); }
    put_u(s, pos, "first_row_indices_without_ending", 0, lr.p, lr.n);
    put_u(s, pos, "first_nz_indices", 0, ln.p, ln.n);
    return 0;
}

/* §8f rank 2: interlance_storage_operator at the GLOBAL parent,
 * modify_{col,val,row}_indices_by_interlance_storage.cc:45-71: all BMTs have
 * BMT_size_of_each_blk nonzeros; the i-th of BMT b moves to b + i * (nnz / size). */
int or_interlance_storage_global(or_set *s) {
    if (!exists(s, "GLOBAL_META", "BMT_size_of_each_blk", 0))
        return fail(s, "interleaved storage needs equal-size BMTs (BMT_size_of_each_blk)");
    uint64_t sz = scalar(s, "GLOBAL_META", "BMT_size_of_each_blk", 0);
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t n = C->len;
    if (sz == 0 || n % sz) return fail(s, "nnz is not a multiple of the BMT size");
    uint64_t nb = n / sz;
    uint64_t *nr = (uint64_t *)malloc(n * sizeof(uint64_t)), *nc = (uint64_t *)malloc(n * sizeof(uint64_t));
    double *nv = (double *)malloc(n * sizeof(double));
    for (uint64_t b = 0; b < nb; b++)
        for (uint64_t i = 0; i < sz; i++) {
            nc[b + i * nb] = C->u[i + b * sz];
            nr[b + i * nb] = R->u[i + b * sz];
            nv[b + i * nb] = V->f[i + b * sz];
        }
    put_u(s, "GLOBAL_META", "nz_col_indices_after_interlance_storage", 0, nc, n);
    put_u(s, "GLOBAL_META", "nz_row_indices_after_interlance_storage", 0, nr, n);
    put_f(s, "GLOBAL_META", "nz_vals_after_interlance_storage", 0, nv, n);
    return 0;
}

/* §8f rank 2 under a TBLOCK / WARP parent (modify_{col,val,row}_indices_by_interlance_storage.cc
 * :73-118): per parent j, spacing = its BMT count n_j, size = its BMT_size_of_each_blk[j],
 * offset = the nonzeros of the parents before it (asserted equal to first_nz_indices[j]);
 * the i-th nonzero of the parent's BMT b moves to offset + b + i * n_j. */
int or_interlance_storage_parent(or_set *s, const char *pos) {
    if (!exists(s, pos, "first_BMT_indices", 0) || !exists(s, pos, "BMT_size_of_each_blk", 0))
        return fail(s, "interleaved storage in a parent needs first_BMT_indices and BMT_size_of_each_blk");
    or_array *F = get(s, pos, "first_BMT_indices", 0), *Z = get(s, pos, "BMT_size_of_each_blk", 0);
    or_array *P = get(s, pos, "first_nz_indices", 0);
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t n = C->len, off = 0;
    uint64_t *nr = (uint64_t *)calloc(n ? n : 1, sizeof(uint64_t)), *nc = (uint64_t *)calloc(n ? n : 1, sizeof(uint64_t));
    double *nv = (double *)calloc(n ? n : 1, sizeof(double));
    for (uint64_t j = 0; j + 1 < F->len; j++) {
        uint64_t nb = F->u[j + 1] - F->u[j], sz = Z->u[j];
        if (P && P->u[j] != off) { free(nr); free(nc); free(nv); return fail(s, "parent first nz != interleaved offset"); }
        if (off + nb * sz > n) { free(nr); free(nc); free(nv); return fail(s, "parent BMTs past the nonzeros"); }
        for (uint64_t b = 0; b < nb; b++)
            for (uint64_t i = 0; i < sz; i++) {
                nc[b + i * nb + off] = C->u[i + b * sz + off];
                nr[b + i * nb + off] = R->u[i + b * sz + off];
                nv[b + i * nb + off] = V->f[i + b * sz + off];
            }
        off += nb * sz;
    }
    put_u(s, "GLOBAL_META", "nz_col_indices_after_interlance_storage", 0, nc, n);
    put_u(s, "GLOBAL_META", "nz_row_indices_after_interlance_storage", 0, nr, n);
    put_f(s, "GLOBAL_META", "nz_vals_after_interlance_storage", 0, nv, n);
    return 0;
}

/* §8f rank 1: model-driven index compression decision (code_generator.cc:16-40 order;
 * if_linear_compress :2618-2640, if_branch_compress :2642-2670, if_cycle_linear_compress
 * :2672-2715, if_cycle_increase_compress :2717-2760, if_residual_compress :2762-2824 and
 * the parameters of the matching get_*_compress).  kind: 0 none, 1 linear, 2 branch,
 * 3 cycle_linear, 4 cycle_increase, 5 residual; params = coef, intercept, cycle, aa, bb;
 * res (n entries, may be NULL) gets the residual array.  Unsigned 64-bit arithmetic. */
static int data_type_of_max(uint64_t m) { /* op_manager.cc:985-1016, struct.hpp enum codes */
    if (m <= 255) return 1;          /* UNSIGNED_CHAR */
    if (m <= 65535) return 6;        /* UNSIGNED_SHORT */
    if (m <= 4294967295ull) return 11; /* UNSIGNED_INT */
    return 16;                       /* UNSIGNED_LONG */
}

int or_index_compression(const uint64_t *a, uint64_t n, int type_ori, int branch_max, int *kind,
                         uint64_t *params, uint64_t *res) {
    for (int i = 0; i < 5; i++) params[i] = 0;
    *kind = 0;
    if (n < 2) return 0;
    /* linear */
    uint64_t coef = a[1] - a[0];
    int ok = 1;
    for (uint64_t i = 0; i + 1 < n && ok; i++)
        if (a[i + 1] - a[i] != coef) ok = 0;
    if (ok) { *kind = 1; params[0] = coef; params[1] = a[0]; return 0; }
    /* branch */
    uint64_t item = a[0], count = 1;
    ok = 1;
    for (uint64_t i = 0; i < n && ok; i++)
        if (a[i] != item) { count++; item = a[i]; if ((int64_t)count >= branch_max) ok = 0; }
    if (ok) { *kind = 2; return 0; }
    /* cycle linear */
    uint64_t icpt = a[0], cyc = 1;
    for (uint64_t i = 1; i < n; i++)
        if (a[i] == icpt) cyc = i;
    ok = 1;
    for (uint64_t i = 0; i < n && ok; i++) {
        uint64_t in = i % cyc;
        if (in == 0 && a[i] != icpt) ok = 0;
        if (in != 0 && (a[i] - icpt) / in != coef) ok = 0;
    }
    if (ok) {
        *kind = 3; params[0] = coef; params[1] = icpt;
        for (uint64_t i = 0; i < n; i++) if (a[i] == icpt) params[2] = i; /* get_: last i >= 0 */
        return 0;
    }
    /* cycle increase */
    cyc = 1;
    ok = 1;
    for (uint64_t i = 1; i < n; i++)
        if (a[i] != a[0]) { if (a[i] < a[0]) ok = 0; cyc = i; break; }
    if (ok && n % cyc != 0) ok = 0;
    for (uint64_t i = 0; i < n && ok; i++) {
        uint64_t id = i / cyc;
        if (id != 0 && (a[i] - a[0]) % id != 0) ok = 0;
    }
    if (ok) {
        *kind = 4; params[1] = a[0];
        for (uint64_t i = 0; i < n; i++)
            if (a[i] != a[0]) { params[2] = i; params[0] = a[i] - a[0]; break; }
        return 0;
    }
    /* residual */
    double t1 = 0, t2 = 0, t3 = 0, t4 = 0, dn = (double)n;
    for (uint64_t i = 0; i < n; i++) {
        t1 += (double)(i * i); t2 += (double)i; t3 += (double)(i * a[i]); t4 += (double)a[i];
    }
    double fa = (t3 * dn - t2 * t4) / (t1 * dn - t2 * t2), fb = (t1 * t4 - t2 * t3) / (t1 * dn - t2 * t2);
    int64_t aa = (int64_t)fa, bb = (int64_t)fb;
    uint64_t m1 = 0, m2 = 0;
    for (uint64_t i = 0; i < n; i++) {
        int64_t e = (int64_t)(a[i] - (uint64_t)aa * i - (uint64_t)bb);
        if (e >= 0) { if ((uint64_t)e > m1) m1 = (uint64_t)e; }
        else if ((uint64_t)(-e) > m2) m2 = (uint64_t)(-e);
    }
    bb -= (int64_t)m2;
    if (data_type_of_max(m1 + m2) < type_ori) {
        *kind = 5; params[3] = (uint64_t)aa; params[4] = (uint64_t)bb;
        if (res) for (uint64_t i = 0; i < n; i++) res[i] = a[i] - (uint64_t)aa * i - (uint64_t)bb;
    }
    return 0;
}

/* §8f rank 1, relative BMW indices inside BMTBs:
 * get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB.cc:45-70 and
 * get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB.cc:50-85
 * (no ending entry; the nz counter restarts at every BMTB) */
int or_bmw_relative_to_bmtb(or_set *s, int rb) {
    or_array *TR = get(s, "TBLOCK_META", "first_row_indices", 0);
    if (!TR || rb < 1) return fail(s, "relative BMW indices need BMTBs");
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    uint64_t row_num = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, row_num);
    vu rr = {0}, rn = {0};
    for (uint64_t i = 0; i + 1 < TR->len; i++) {
        uint64_t b = TR->u[i], e = TR->u[i + 1], nz = 0;
        for (uint64_t r = b; r < e; r += (uint64_t)rb) vu_push(&rr, r - b);
        for (uint64_t r = b; r < e; r++) {
            if ((r - b) % (uint64_t)rb == 0) vu_push(&rn, nz);
            nz += r < row_num ? cnt[r] : 0;
        }
    }
    free(cnt);
    put_u(s, "WARP_META", "first_row_indices_relative_to_BMTB", 0, rr.p, rr.n);
    put_u(s, "WARP_META", "first_nz_indices_relative_to_BMTB", 0, rn.p, rn.n);
    return 0;
}

/* ------------------------------------------------------------------ */
/* canned pipelines: token_test.cc test_spmm_*                          */
/* ------------------------------------------------------------------ */

/* §8f rank 1: BMT row blocking inside the BMWs (else the BMTBs), fixed_interval_row_direction_
 * thread_blocking_operator.cc:198-480 with get_begin_{rows,nzs}_of_BMT_after_fixed_blocking_in_
 * row_direction_{in,relative_to}_{BMTB,BMW}.cc and get_begin_BMTs_of_specific_parent_after_blocking_
 * in_row_direction.cc.  Rows: BMTs start at first + k*rb inside each parent (+ row_num at the
 * end; relative: minus the parent's first row, no end).  Nzs: each parent opens a BMT at its
 * first nz, a new one after every rb rows that do not end the parent (+ the parents' last nz;
 * relative: from 0, no end).  Parent first_BMT_indices: BMTs per parent, prefix-summed. */
int or_bmt_in_parent(or_set *s, int rb, int rrel, int nrel) {
    const char *pp = get(s, "WARP_META", "first_row_indices", 0) ? "WARP_META" : "TBLOCK_META";
    const char *tag = pp[0] == 'W' ? "BMW" : "BMTB";
    or_array *PR = get(s, pp, "first_row_indices", 0), *PZ = get(s, pp, "first_nz_indices", 0);
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    if (!PR || !PZ || !R || rb < 1) return fail(s, "BMT blocking in a parent needs BMTB/BMW row blocks");
    uint64_t rn = row_num_of(s);
    uint64_t *cnt = row_nnz(R->u, R->len, rn);
    vu ar = {0}, rr = {0}, az = {0}, rz = {0}, pb = {0};
    vu_push(&pb, 0);
    for (uint64_t j = 0; j + 1 < PR->len; j++) {
        uint64_t f = PR->u[j], nx = PR->u[j + 1], nbmt = 0;
        for (uint64_t r = f; r < nx; r += (uint64_t)rb) {
            vu_push(&ar, r);
            vu_push(&rr, r - f);
            nbmt++;
        }
        uint64_t rc = 0, nz = 0;
        vu_push(&az, PZ->u[j]);
        vu_push(&rz, 0);
        for (uint64_t i = f; i < nx; i++) {
            rc++;
            nz += cnt[i];
            if (rc == (uint64_t)rb && i != nx - 1) {
                vu_push(&az, PZ->u[j] + nz);
                vu_push(&rz, nz);
                rc = 0;
            }
        }
        vu_push(&pb, pb.p[pb.n - 1] + nbmt);
    }
    free(cnt);
    vu_push(&ar, rn);
    vu_push(&az, PZ->u[PZ->len - 1]);
    char k1[64], k2[64];
    snprintf(k1, sizeof k1, "first_row_indices_relative_to_%s", tag);
    snprintf(k2, sizeof k2, "first_nz_indices_relative_to_%s", tag);
    put_u(s, "THREAD_META", "first_row_indices", 0, ar.p, ar.n);
    if (rrel) put_u(s, "THREAD_META", k1, 0, rr.p, rr.n);
    else free(rr.p);
    put_u(s, "THREAD_META", "first_nz_indices", 0, az.p, az.n);
    if (nrel) put_u(s, "THREAD_META", k2, 0, rz.p, rz.n);
    else free(rz.p);
    put_u(s, pp, "first_BMT_indices", 0, pb.p, pb.n);
    return 0;
}

/* §8f rank 3: fixed_interval_row_matrix_div_operator on sub-matrix 0
 * (operator/fixed_interval_row_matrix_div_operator.cc:61-150 validity + run order;
 * transform_step/modify_{row,col}_{start,end}_boundary_after_fixed_div_in_row_direction.cc,
 * fixed_div_{col_indices_by_corr_row_indices,vals_by_corr_row_indices,row_indices}.cc).
 * Interval i = rows [begin + i*gap, begin + (i+1)*gap - 1] (the end clamped to
 * end_row_index); every non-empty interval becomes sub-matrix (max id + 1), in interval
 * order, holding its nonzeros in their order with rows reduced modulo gap; sub-matrix
 * 0's row / col / val arrays are removed (its boundaries stay). */
int or_fixed_interval_row_div(or_set *s, uint64_t gap) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    if (!R || !C || !V || gap == 0) return fail(s, "row division needs the COO of sub-matrix 0 and gap > 0");
    if (exists(s, "GLOBAL_META", "nz_col_indices_after_interlance_storage", 0))
        return fail(s, "row division after interleaved storage");
    uint64_t b = scalar(s, "GLOBAL_META", "begin_row_index", 0), e = scalar(s, "GLOBAL_META", "end_row_index", 0);
    uint64_t bc = scalar(s, "GLOBAL_META", "begin_col_index", 0), ec = scalar(s, "GLOBAL_META", "end_col_index", 0);
    uint64_t row_num = e - b + 1, nbin = (row_num + gap - 1) / gap;
    uint64_t *cnt = (uint64_t *)calloc(nbin ? nbin : 1, sizeof(uint64_t));
    uint64_t non_empty = 0;
    for (uint64_t i = 0; i < R->len; i++) {
        if (R->u[i] / gap >= nbin) {
            free(cnt);
            return fail(s, "row division: a nonzero past end_row_index");
        }
        if (cnt[R->u[i] / gap]++ == 0) non_empty++;
    }
    if (!(row_num > gap) || non_empty > 12) { /* MAX_DIV_TIMES_OF_DIV default */
        free(cnt);
        return fail(s, "row division invalid: %llu rows, gap %llu, %llu intervals", (unsigned long long)row_num,
                    (unsigned long long)gap, (unsigned long long)non_empty);
    }
    int id = 1; /* sub-matrix 0 is the only one before the division */
    for (uint64_t bin = 0; bin < nbin; bin++) {
        if (!cnt[bin]) continue;
        uint64_t n = cnt[bin], k = 0;
        uint64_t *nr = (uint64_t *)malloc(n * sizeof(uint64_t)), *nc = (uint64_t *)malloc(n * sizeof(uint64_t));
        double *nv = (double *)malloc(n * sizeof(double));
        for (uint64_t i = 0; i < R->len; i++)
            if (R->u[i] / gap == bin) {
                nr[k] = R->u[i] % gap;
                nc[k] = C->u[i];
                nv[k] = V->f[i];
                k++;
            }
        uint64_t hi = b + (bin + 1) * gap - 1;
        put_scalar(s, "GLOBAL_META", "begin_row_index", id, b + bin * gap);
        put_scalar(s, "GLOBAL_META", "end_row_index", id, hi >= e ? e : hi);
        put_scalar(s, "GLOBAL_META", "begin_col_index", id, bc);
        put_scalar(s, "GLOBAL_META", "end_col_index", id, ec);
        put_u(s, "GLOBAL_META", "nz_col_indices", id, nc, n);
        put_f(s, "GLOBAL_META", "nz_vals", id, nv, n);
        put_u(s, "GLOBAL_META", "nz_row_indices", id, nr, n);
        R = get(s, "GLOBAL_META", "nz_row_indices", 0); /* put_* may move entries */
        C = get(s, "GLOBAL_META", "nz_col_indices", 0);
        V = get(s, "GLOBAL_META", "nz_vals", 0);
        id++;
    }
    free(cnt);
    drop(s, "GLOBAL_META", "nz_col_indices", 0);
    drop(s, "GLOBAL_META", "nz_vals", 0);
    drop(s, "GLOBAL_META", "nz_row_indices", 0);
    return 0;
}

/* §8f rank 3: row_nz_matrix_div_operator on sub-matrix 0 (operator/row_nz_matrix_div_operator.cc
 * :59-250; transform_step/modify_*_boundary_after_div_according_to_row_nz.cc,
 * div_{row,col,val}_indices_by_row_nnz.cc).
 * Window of a row length nz: [0, init) grown by rate while nz >= high and high <= max_gap;
 * nz >= max_gap gives [max_gap, max_gap*rate).  A division position is every row whose
 * length leaves the current window (lengths past an open-ended top window stay).  Every
 * position gets boundaries (begin = position, end = next position - 1, cols copied); the
 * entries walk the buckets in row order, moving on by one bucket whenever a row reaches the
 * current bucket's bound (the last bucket's bound: last row + 1); only non-empty buckets get
 * arrays; rows keep sub-matrix 0's indexing. */
static void rnz_window(uint64_t nz, uint64_t init, uint64_t mx, uint64_t rate, uint64_t *lo, uint64_t *hi) {
    *lo = 0;
    *hi = init;
    if (nz < mx) {
        while (nz >= *hi && *hi <= mx) {
            *lo = *hi;
            *hi *= rate;
        }
    } else {
        *lo = mx;
        *hi = mx * rate;
    }
}

int or_row_nz_div(or_set *s, uint64_t init, uint64_t mx, uint64_t rate) {
    or_array *R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    or_array *C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    or_array *V = get(s, "GLOBAL_META", "nz_vals", 0);
    if (!R || !C || !V || !R->len || init == 0 || rate == 0) return fail(s, "row-length division needs the COO of sub-matrix 0");
    uint64_t b = scalar(s, "GLOBAL_META", "begin_row_index", 0), e = scalar(s, "GLOBAL_META", "end_row_index", 0);
    uint64_t bc = scalar(s, "GLOBAL_META", "begin_col_index", 0), ec = scalar(s, "GLOBAL_META", "end_col_index", 0);
    uint64_t rn = e - b + 1;
    uint64_t *cnt = row_nnz(R->u, R->len, rn);
    uint64_t *div = (uint64_t *)malloc((rn + 1) * sizeof(uint64_t));
    uint64_t nd = 0, lo, hi;
    div[nd++] = 0;
    rnz_window(cnt[0], init, mx, rate, &lo, &hi);
    for (uint64_t r = 1; r < rn; r++) {
        uint64_t nz = cnt[r];
        if ((nz >= lo && nz < hi) || (nz >= hi && hi > mx)) continue;
        div[nd++] = r;
        if (nd > 12) { /* MAX_DIV_TIMES_OF_DIV default */
            free(cnt);
            free(div);
            return fail(s, "row-length division: more than 12 positions");
        }
        rnz_window(nz, init, mx, rate, &lo, &hi);
    }
    free(cnt);
    int id = 1;
    for (uint64_t i = 0; i < nd; i++) {
        put_scalar(s, "GLOBAL_META", "begin_row_index", (int)(id + i), div[i]);
        put_scalar(s, "GLOBAL_META", "end_row_index", (int)(id + i), (i + 1 < nd ? div[i + 1] : rn) - 1);
        put_scalar(s, "GLOBAL_META", "begin_col_index", (int)(id + i), bc);
        put_scalar(s, "GLOBAL_META", "end_col_index", (int)(id + i), ec);
    }
    R = get(s, "GLOBAL_META", "nz_row_indices", 0);
    C = get(s, "GLOBAL_META", "nz_col_indices", 0);
    V = get(s, "GLOBAL_META", "nz_vals", 0);
    uint64_t n = R->len, last = R->u[n - 1];
    uint64_t *bk = (uint64_t *)malloc(n * sizeof(uint64_t)), *bn = (uint64_t *)calloc(nd, sizeof(uint64_t));
    uint64_t cur = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r = R->u[i], up = cur < nd - 1 ? div[cur + 1] : last + 1;
        if (r >= up) cur++;
        bk[i] = cur;
        bn[cur]++;
    }
    free(div);
    int nid = id;
    for (uint64_t k = 0; k < nd; k++) {
        if (!bn[k]) continue;
        uint64_t *nr = (uint64_t *)malloc(bn[k] * sizeof(uint64_t)), *nc = (uint64_t *)malloc(bn[k] * sizeof(uint64_t));
        double *nv = (double *)malloc(bn[k] * sizeof(double));
        uint64_t q = 0;
        for (uint64_t i = 0; i < n; i++)
            if (bk[i] == k) {
                nr[q] = R->u[i];
                nc[q] = C->u[i];
                nv[q] = V->f[i];
                q++;
            }
        put_u(s, "GLOBAL_META", "nz_col_indices", nid, nc, bn[k]);
        put_f(s, "GLOBAL_META", "nz_vals", nid, nv, bn[k]);
        put_u(s, "GLOBAL_META", "nz_row_indices", nid, nr, bn[k]);
        R = get(s, "GLOBAL_META", "nz_row_indices", 0);
        C = get(s, "GLOBAL_META", "nz_col_indices", 0);
        V = get(s, "GLOBAL_META", "nz_vals", 0);
        nid++;
    }
    free(bk);
    free(bn);
    drop(s, "GLOBAL_META", "nz_col_indices", 0);
    drop(s, "GLOBAL_META", "nz_vals", 0);
    drop(s, "GLOBAL_META", "nz_row_indices", 0);
    return 0;
}

int or_pipeline(or_set *s, const char *name, int p0, int p1) {
    if (!strcmp(name, "tblock_thread_total")) { /* BMTB rows p0, BMT rows p1 inside them (relative too) */
        if (or_row_dir_tblock_blocking(s, p0)) return -1;
        return or_bmt_in_parent(s, p1 > 0 ? p1 : 1, 1, 1);
    }
    if (!strcmp(name, "tblock_balanced_thread_total")) { /* BMTBs of p0 rows, balanced BMTs of p1 nnz inside */
        if (or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 64)) return -1;
        return or_balanced_in_parent(s, p1 > 0 ? (uint64_t)p1 : 64, 1, "THREAD_META", "TBLOCK_META", "BMTB",
                                     "first_BMT_indices");
    }
    if (!strcmp(name, "tblock_balanced_warp_total")) { /* BMTBs of p0 rows, balanced BMWs of p1 nnz inside */
        if (or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 64)) return -1;
        return or_balanced_bmw_in_bmtb(s, p1 > 0 ? (uint64_t)p1 : 256, 1);
    }
    if (!strcmp(name, "tblock_thread_total_maxpad")) { /* every row (empty ones too) to its BMTB's longest */
        if (col_pad_max(s, p0 > 0 ? (uint64_t)p0 : 16, 1)) return -1;
        if (or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 16)) return -1;
        return or_bmt_in_parent(s, p1 > 0 ? p1 : 1, 1, 1);
    }
    if (!strcmp(name, "tblock_thread_total_colpad")) { /* BMTs of one row in BMTBs of p0 rows, rows to a multiple of p1 */
        if (col_pad(s, p1 > 1 ? p1 : 2)) return -1;
        if (or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 16)) return -1;
        return or_bmt_in_parent(s, 1, 1, 1);
    }
    if (!strcmp(name, "thread_total_maxpad")) { /* ELL-like: every row to the longest, BMTs of p0 rows */
        if (col_pad_max(s, 0, 1)) return -1;
        return or_row_dir_thread_blocking(s, p0 > 0 ? p0 : 1, 0);
    }
    if (!strcmp(name, "tblock_warp_thread_total")) { /* BMTB rows p0, BMW rows 8, BMT rows p1 in the BMWs */
        if (or_row_dir_tblock_blocking(s, p0)) return -1;
        if (or_row_dir_warp_blocking(s, 8)) return -1;
        return or_bmt_in_parent(s, p1 > 0 ? p1 : 1, 1, 1);
    }
    if (!strcmp(name, "row_div")) /* p0 = fixed_row_interval_size */
        return or_fixed_interval_row_div(s, (uint64_t)p0);
    if (!strcmp(name, "row_nz_div")) /* p0 = init window, p1 = max window; expansion rate 2 */
        return or_row_nz_div(s, (uint64_t)p0, (uint64_t)p1, 2);
    if (!strcmp(name, "empty_row_pad")) return or_empty_row_pad(s);
    if (!strncmp(name, "empty_pad_", 10)) { /* empty_row_pad_operator, then the named sequence */
        if (or_empty_row_pad(s)) return -1;
        return or_pipeline(s, name + 10, p0, p1);
    }
    if (!strcmp(name, "thread_total")) { /* token_test.cc:1003-1092, p0 = sparse_cf */
        if (or_sort_operator(s)) return -1;
        return or_row_dir_thread_blocking(s, 1, p0);
    }
    if (!strcmp(name, "warp_total")) /* token_test.cc:1188-1249 */
        return or_row_dir_warp_blocking(s, 1);
    if (!strcmp(name, "block_total_rowpad")) { /* BMTBs of p0 rows, the rows padded to a multiple of p0 */
        if (row_pad(s, p0 > 0 ? p0 : 1)) return -1;
        return or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 1);
    }
    if (!strcmp(name, "warp_total_rowpad")) { /* BMWs of p0 rows, padded likewise */
        if (row_pad(s, p0 > 0 ? p0 : 1)) return -1;
        return or_row_dir_warp_blocking(s, p0 > 0 ? p0 : 1);
    }
    if (!strcmp(name, "block_total")) /* token_test.cc:1458-1514 (rb 1 there; p0 = rows per BMTB) */
        return or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 1);
    /* nnz-direction parents (p0 = nnz per BMW / BMTB, p1 = nnz per BMW inside the BMTBs),
     * padded at the outer level, 32-nnz BMTs inside (relative indices), thread bitmaps of
     * VW 32 (N >= 32) */
    /* col-direction parents: BMWs / BMTBs of p0 nonzeros of a row (tblock_col_warp_total: BMWs
     * of p1 nonzeros inside row-direction BMTBs of p0 rows, relative indices), and col-direction
     * BMTs of p1 nonzeros inside row-direction BMTBs / BMWs of p0 rows (relative indices) */
    if (!strcmp(name, "col_warp_total")) return or_col_dir_warp_blocking(s, p0 > 0 ? (uint64_t)p0 : 64, 0, 0);
    if (!strcmp(name, "col_tblock_total")) return or_col_dir_tblock_blocking(s, p0 > 0 ? (uint64_t)p0 : 256, 0);
    if (!strcmp(name, "tblock_col_warp_total")) {
        if (or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 16)) return -1;
        return or_col_dir_warp_blocking(s, p1 > 0 ? (uint64_t)p1 : 64, 1, 1);
    }
    if (!strcmp(name, "tblock_col_thread_maxpad") || !strcmp(name, "warp_col_thread_maxpad")) {
        /* every non-empty row padded to its BMTB's (BMW's) longest row, then BMTs of p1 in it */
        int warp = !strcmp(name, "warp_col_thread_maxpad");
        uint64_t rb = p0 > 0 ? (uint64_t)p0 : 16, c = p1 > 0 ? (uint64_t)p1 : 32;
        if (col_pad_max(s, rb, 0)) return -1;
        if (warp ? or_row_dir_warp_blocking(s, (int)rb) : or_row_dir_tblock_blocking(s, (int)rb)) return -1;
        return or_col_dir_thread_in_parent(s, c, 1, 1, 0);
    }
    if (!strcmp(name, "tblock_col_thread_interleaved") || !strcmp(name, "warp_col_thread_interleaved")) {
        /* the padded plan + interleave per BMTB (per BMW) */
        int warp = !strcmp(name, "warp_col_thread_interleaved");
        uint64_t c = p1 > 0 ? (uint64_t)p1 : 32;
        if (col_pad(s, (int)c)) return -1;
        if (warp ? or_row_dir_warp_blocking(s, p0 > 0 ? p0 : 16) : or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 16)) return -1;
        if (or_col_dir_thread_in_parent(s, c, 1, 1, 1)) return -1;
        return or_interlance_storage_parent(s, warp ? "WARP_META" : "TBLOCK_META");
    }
    if (!strcmp(name, "tblock_col_thread_total") || !strcmp(name, "warp_col_thread_total") ||
        !strcmp(name, "tblock_col_thread_total_padded")) {
        int pad = !strcmp(name, "tblock_col_thread_total_padded");
        uint64_t c = p1 > 0 ? (uint64_t)p1 : 32;
        if (pad && col_pad(s, (int)c)) return -1;
        if (!strcmp(name, "warp_col_thread_total")) {
            if (or_row_dir_warp_blocking(s, p0 > 0 ? p0 : 16)) return -1;
        } else if (or_row_dir_tblock_blocking(s, p0 > 0 ? p0 : 16)) return -1;
        return or_col_dir_thread_in_parent(s, c, 1, 1, pad);
    }
    if (!strcmp(name, "nnz_warp_bitmap")) {
        if (or_nnz_dir_warp_blocking(s, (uint64_t)p0, 0, 0, 1)) return -1;
        if (or_nnz_dir_thread_in_parent(s, 32, 1, 1)) return -1;
        return or_thread_bit_map_operator(s, 0, 32);
    }
    if (!strcmp(name, "nnz_tblock_bitmap")) {
        if (or_nnz_dir_tblock_blocking(s, (uint64_t)p0, 1)) return -1;
        if (or_nnz_dir_thread_in_parent(s, 32, 1, 1)) return -1;
        return or_thread_bit_map_operator(s, 0, 32);
    }
    if (!strcmp(name, "nnz_tblock_warp_bitmap")) {
        if (or_nnz_dir_tblock_blocking(s, (uint64_t)p0, 1)) return -1;
        if (or_nnz_dir_warp_blocking(s, (uint64_t)p1, 1, 1, 0)) return -1;
        if (or_nnz_dir_thread_in_parent(s, 32, 1, 1)) return -1;
        return or_thread_bit_map_operator(s, 0, 32);
    }
    if (!strcmp(name, "thread_bit_map")) { /* token_test.cc:1319-1391, p0 = VW */
        if (or_nnz_dir_thread_blocking(s, 32, 1)) return -1;
        return or_thread_bit_map_operator(s, 0, p0);
    }
    if (!strcmp(name, "warp_segment")) { /* token_test.cc:1393-1455, p0 = VW */
        if (or_nnz_dir_thread_blocking(s, 32, 1)) return -1;
        if (or_thread_bit_map_operator(s, 1, p0)) return -1;
        return or_warp_segment_operator(s, p0);
    }
    if (!strcmp(name, "tblock_warp_total")) { /* tblock rows p0 + BMW rows p1 (default 1) + warp_total */
        if (or_row_dir_tblock_blocking(s, p0)) return -1;
        return or_row_dir_warp_blocking(s, p1 > 0 ? p1 : 1);
    }
    if (!strcmp(name, "warp_bit_map")) { /* token_test.cc:1250-1315, p0 = VW = max(128/min(N/cf,32), 32) */
        if (or_col_dir_thread_blocking(s, 64, 1)) return -1;
        return or_parent_bit_map_operator(s, 1, p0, 1, 1);
    }
    if (!strcmp(name, "tblock_bit_map")) { /* token_test.cc:1515-1582, p0 = block_size = 256/min(N/cf,32) */
        if (or_col_dir_thread_blocking(s, 64, 1)) return -1;
        return or_parent_bit_map_operator(s, 0, p0, 0, 0);
    }
    if (!strcmp(name, "warp_bit_map_interleaved")) { /* §8f rank 2 on the warp_bit_map plan */
        if (or_col_dir_thread_blocking(s, 64, 1)) return -1;
        if (or_interlance_storage_global(s)) return -1;
        return or_parent_bit_map_operator(s, 1, p0, 1, 1);
    }
    if (!strcmp(name, "tblock_bit_map_interleaved")) {
        if (or_col_dir_thread_blocking(s, 64, 1)) return -1;
        if (or_interlance_storage_global(s)) return -1;
        return or_parent_bit_map_operator(s, 0, p0, 0, 0);
    }
    if (!strcmp(name, "tblock_warp_total_relative")) { /* BMW indices relative to the BMTB too */
        if (or_row_dir_tblock_blocking(s, p0)) return -1;
        if (or_row_dir_warp_blocking(s, p1 > 0 ? p1 : 1)) return -1;
        return or_bmw_relative_to_bmtb(s, p1 > 0 ? p1 : 1);
    }
    if (!strcmp(name, "balanced_warp_total")) /* A11 balanced BMW + warp_total */
        return or_balanced_row_dir_warp_blocking(s, (uint64_t)p0);
    if (!strcmp(name, "balanced_block_total")) /* A11 balanced BMTB + tblock_total */
        return or_balanced_row_dir_tblock_blocking(s, (uint64_t)(p0 > 0 ? p0 : 4096));
    if (!strcmp(name, "balanced_thread_total")) /* A11 balanced BMT + thread_total */
        return or_balanced_row_dir_thread_blocking(s, (uint64_t)(p0 > 0 ? p0 : 64));
    if (!strcmp(name, "merge_path")) /* A11 merge path; p1: 0/1 WARP, 2 TBLOCK, 3 THREAD */
        return or_merge_path(s, p1 == 2 ? "TBLOCK_META" : (p1 == 3 ? "THREAD_META" : "WARP_META"),
                             (uint64_t)(p0 > 0 ? p0 : 1024));
    return fail(s, "unknown pipeline %s", name);
}

/* ------------------------------------------------------------------ */
/* A17: CPU SpMM references                                             */
/* ------------------------------------------------------------------ */

void or_spmm_f64(uint64_t M, uint64_t N, uint64_t nnz, const uint64_t *row,
                 const uint64_t *col, const float *val, const double *B,
                 double *C) {
    memset(C, 0, M * N * sizeof(double));
    for (uint64_t p = 0; p < nnz; p++) {
        double v = val[p];
        const double *b = B + col[p] * N;
        double *c = C + row[p] * N;
        for (uint64_t j = 0; j < N; j++) c[j] += v * b[j];
    }
}

/* kernel_lib.hpp:859-881: per row, products added in CSR order */
void or_spmm_ref_f32(uint64_t M, uint64_t N, uint64_t nnz, const uint64_t *row,
                     const uint64_t *col, const float *val, const float *B,
                     float *C) {
    memset(C, 0, M * N * sizeof(float));
    for (uint64_t p = 0; p < nnz; p++) {
        float v = val[p];
        const float *b = B + col[p] * N;
        float *c = C + row[p] * N;
        for (uint64_t j = 0; j < N; j++) c[j] += v * b[j];
    }
}

/* IEEE binary16 round-to-nearest-even, via bit manipulation */
float or_round_half(float x) {
    union { float f; uint32_t u; } in = {x};
    uint32_t u = in.u, sign = u & 0x80000000u;
    uint32_t a = u & 0x7fffffffu;
    if (a >= 0x7f800000u) return x; /* inf / nan */
    float ax;
    union { uint32_t u; float f; } t = {a};
    ax = t.f;
    if (ax >= 65520.0f) { union { uint32_t u; float f; } r = {sign | 0x7f800000u}; return r.f; }
    if (ax < 6.103515625e-05f) { /* subnormal half: quantum 2^-24 */
        float q = 5.9604644775390625e-08f;
        float r = nearbyintf(ax / q) * q;
        union { float f; uint32_t u; } o = {r};
        o.u |= sign;
        return o.f;
    }
    /* normal: keep 10 mantissa bits */
    uint32_t lsb = (a >> 13) & 1u;
    uint32_t rounded = (a + 0x0fffu + lsb) & ~0x1fffu;
    union { uint32_t u; float f; } o = {rounded | sign};
    return o.f;
}

void or_spmm_ref_f16(uint64_t M, uint64_t N, uint64_t nnz, const uint64_t *row,
                     const uint64_t *col, const float *val, const float *B,
                     float *C) {
    memset(C, 0, M * N * sizeof(float));
    for (uint64_t p = 0; p < nnz; p++) {
        float v = or_round_half(val[p]);
        const float *b = B + col[p] * N;
        float *c = C + row[p] * N;
        for (uint64_t j = 0; j < N; j++)
            c[j] = or_round_half(c[j] + or_round_half(v * or_round_half(b[j])));
    }
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int or_time_cpu_path(uint64_t M, uint64_t K, uint64_t nnz, const uint64_t *row,
                     const uint64_t *col, const float *val, uint64_t N,
                     double *t_transform, double *t_spmm) {
    or_set s;
    double t0 = now_s();
    if (or_init_set(&s, M, K, nnz, row, col, val)) return -1;
    if (or_pipeline(&s, "thread_total", 4, 0)) { or_set_free(&s); return -1; }
    double t1 = now_s();
    or_set_free(&s);
    float *B = (float *)malloc(K * N * sizeof(float));
    float *C = (float *)malloc(M * N * sizeof(float));
    for (uint64_t i = 0; i < K * N; i++) B[i] = 1.0f;
    double t2 = now_s();
    or_spmm_ref_f32(M, N, nnz, row, col, val, B, C);
    double t3 = now_s();
    volatile float sink = C[0];
    (void)sink;
    free(B); free(C);
    *t_transform = t1 - t0;
    *t_spmm = t3 - t2;
    return 0;
}

/* CPU baseline leg of bench.py: the host SpMM (spmm_reference_host restated,
 * fp32) repeated until at least min_s seconds of work, single thread. */
int or_time_spmm_repeated(uint64_t M, uint64_t K, uint64_t nnz, const uint64_t *row,
                          const uint64_t *col, const float *val, uint64_t N, double min_s,
                          double *t_total, int *reps) {
    float *B = (float *)malloc(K * N * sizeof(float));
    float *C = (float *)malloc(M * N * sizeof(float));
    if (!B || !C) { free(B); free(C); return -1; }
    for (uint64_t i = 0; i < K * N; i++) B[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
    int r = 0;
    double t0 = now_s(), t = 0;
    do {
        or_spmm_ref_f32(M, N, nnz, row, col, val, B, C);
        r++;
        t = now_s() - t0;
    } while (t < min_s);
    volatile float sink = C[0];
    (void)sink;
    free(B); free(C);
    *t_total = t;
    *reps = r;
    return 0;
}

/* The build's all-cores variant of the host SpMM (NOT the reference's: its host path is
 * single-threaded): the same fp32 products and row sums over a CSR of the
 * row-sorted COO, rows split over `threads` OpenMP threads.  Timed like
 * or_time_spmm_repeated. */
int or_time_spmm_repeated_mt(uint64_t M, uint64_t K, uint64_t nnz, const uint64_t *row,
                             const uint64_t *col, const float *val, uint64_t N, double min_s,
                             int threads, double *t_total, int *reps) {
    float *B = (float *)malloc(K * N * sizeof(float));
    float *C = (float *)malloc(M * N * sizeof(float));
    uint64_t *rp = (uint64_t *)calloc(M + 1, sizeof(uint64_t));
    if (!B || !C || !rp) { free(B); free(C); free(rp); return -1; }
    for (uint64_t i = 0; i < K * N; i++) B[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
    for (uint64_t p = 0; p < nnz; p++) {
        if (row[p] >= M || (p && row[p] < row[p - 1])) { free(B); free(C); free(rp); return -2; }
        rp[row[p] + 1]++;
    }
    for (uint64_t i = 0; i < M; i++) rp[i + 1] += rp[i];
    int r = 0;
    double t0 = now_s(), t = 0;
    do {
#pragma omp parallel for num_threads(threads) schedule(dynamic, 64)
        for (int64_t i = 0; i < (int64_t)M; i++) {
            float *c = C + (uint64_t)i * N;
            for (uint64_t j = 0; j < N; j++) c[j] = 0.f;
            for (uint64_t p = rp[i]; p < rp[i + 1]; p++) {
                const float v = val[p];
                const float *b = B + col[p] * N;
                for (uint64_t j = 0; j < N; j++) c[j] += v * b[j];
            }
        }
        r++;
        t = now_s() - t0;
    } while (t < min_s);
    volatile float sink = C[0];
    (void)sink;
    free(B); free(C); free(rp);
    *t_total = t;
    *reps = r;
    return 0;
}
