/*
 * ora_pipeline.c -- plain-C restatement of AntiZ's precompress/reconstruct pipeline
 * (TEST INFRASTRUCTURE ONLY; cites /root/reference/main.cpp line numbers).
 *
 *  Phase 1  ora_scan       ATZcreator::searchInfile main.cpp:392-420, ZBuffSearcher main.cpp:149-249
 *  Phase 3  ora_sweep      findDeflateParams_ALL/_stream, tryParams*, testParamRange,
 *                          testDeflateParams, deltaEncode  main.cpp:421-763
 *  Phase 4  ora_write_atz  writeATZfile/writeStreamdesc main.cpp:764-834 (ATZ1 layout SURVEY.md App. C)
 *  -r       ora_reconstruct ATZreconstructor main.cpp:862-1064
 *
 * Chunk buffers are rebuilt exactly as searchInfile builds them, including its off-by-one:
 * for chunks >= 1 the carried byte is rBuffer[gcount-1] (main.cpp:413), i.e. the SECOND-TO-LAST
 * byte of the data just read, so from the third chunk on buffer[0] is not the file byte at
 * chunkOffset.  A stream still being inflated at a chunk end is continued with the next buffer
 * (main.cpp:207-217); since zlib had consumed every byte offered, that equals inflating the
 * concatenation of the offered buffers from scratch, which is what this code does.
 */
#include "atz_oracle.h"
#include <stdlib.h>
#include <string.h>

static int parse_type(unsigned h) { /* main.cpp:168-203 */
    static const uint16_t H[24] = {0x2815, 0x2853, 0x2891, 0x28cf, 0x3811, 0x384f, 0x388d, 0x38cb,
                                   0x480d, 0x484b, 0x4889, 0x48c7, 0x5809, 0x5847, 0x5885, 0x58c3,
                                   0x6805, 0x6843, 0x6881, 0x68de, 0x7801, 0x785e, 0x789c, 0x78da};
    for (int t = 0; t < 24; t++) if (H[t] == h) return t;
    return -1;
}

typedef struct {
    ora_stream_t *v; uint64_t n, cap;
} svec;
static int push(svec *s, uint64_t off, int type, uint64_t cl, uint64_t il) {
    if (s->n == s->cap) {
        uint64_t nc = s->cap ? 2 * s->cap : 256;
        ora_stream_t *p = (ora_stream_t *)realloc(s->v, nc * sizeof(*p));
        if (!p) return -1;
        s->v = p; s->cap = nc;
    }
    ora_stream_t *r = &s->v[s->n++];
    memset(r, 0, sizeof(*r));
    r->offset = off; r->type = type; r->comp_len = cl; r->infl_len = il;
    r->clevel = 9; r->window = 15; r->memlevel = 9;   /* streamOffset ctor, ATZData.h:46-58 */
    r->first_diff = -1;
    return 0;
}

typedef struct {
    int need_more;
    uint64_t last_chunk_off, chunk_off;
    int type;
    /* pending inflater: every byte offered since its reset, and its state */
    uint8_t *pend; uint64_t pend_len, pend_cap;
    int pend_state;   /* ORA_INF_* of the last call */
    uint64_t pend_in, pend_out;
} searcher;

static int pend_append(searcher *z, const uint8_t *b, uint64_t n) {
    if (z->pend_len + n > z->pend_cap) {
        uint64_t nc = (z->pend_len + n) * 2;
        uint8_t *p = (uint8_t *)realloc(z->pend, nc);
        if (!p) return -1;
        z->pend = p; z->pend_cap = nc;
    }
    memcpy(z->pend + z->pend_len, b, n);
    z->pend_len += n;
    return 0;
}

/* ZBuffSearcher::operator(), main.cpp:205-246 */
static int search_chunk(searcher *z, const uint8_t *buf, uint64_t len, svec *out) {
    uint64_t i = 0, redlen = len - 1;
    if (z->need_more) {
        uint64_t avail_in;
        int ret;
        if (z->pend_state == ORA_INF_NEED_INPUT) {
            uint64_t before = z->pend_len;
            if (pend_append(z, buf, len)) return -1;
            uint64_t c, p;
            z->pend_state = ora_inflate(z->pend, z->pend_len, NULL, 0, &c, &p);
            z->pend_in = c; z->pend_out = p;
            avail_in = z->pend_len - c;
            (void)before;
            ret = z->pend_state;
        } else if (z->pend_state == ORA_INF_END) {  /* inflate() in DONE mode: Z_STREAM_END again */
            avail_in = len; ret = ORA_INF_END;
        } else {                                    /* BAD mode: Z_DATA_ERROR, nothing consumed */
            avail_in = len; ret = ORA_INF_ERROR;
        }
        if (ret == ORA_INF_END) {
            if (push(out, z->last_chunk_off, z->type, z->pend_in, z->pend_out)) return -1;
            i = len - avail_in;
        }
        z->need_more = (avail_in == 0);
    }
    for (; i < redlen && !z->need_more; i++) {
        unsigned header = (unsigned)buf[i] * 256u + buf[i + 1];
        z->type = parse_type(header);
        if (z->type >= 0) {
            uint64_t c, p;
            int st = ora_inflate(buf + i, len - i, NULL, 0, &c, &p);
            if (c <= 16) continue;
            if (st == ORA_INF_END) {
                if (push(out, i + z->chunk_off, z->type, c, p)) return -1;
                i += c;
                i--;
            } else if ((z->need_more = (c == len - i))) {
                z->last_chunk_off = i + z->chunk_off;
                z->pend_len = 0;
                if (pend_append(z, buf + i, len - i)) return -1;
                z->pend_state = st; z->pend_in = c; z->pend_out = p;
            }
        }
    }
    z->chunk_off += redlen;
    return 0;
}

int ora_scan(const uint8_t *file, uint64_t n, uint64_t cs, ora_result_t *res) {
    memset(res, 0, sizeof(*res));
    if (cs < 2) return -2;              /* reference loops forever at cs==1 (main.cpp:410-415) */
    if (n == 0) return -21;             /* reference reads rBuffer[-1] (main.cpp:406) and crashes (tests/golden/fuzz_small.json: rc -11): UB, reported as the library does (ATZ_E_REF_UB) */
    svec out = {0};
    searcher z;
    memset(&z, 0, sizeof(z));
    uint8_t *rb = (uint8_t *)malloc(cs);
    if (!rb) return -1;
    uint64_t pos = 0;
    uint64_t g = n < cs ? n : cs;                       /* chunk 0: main.cpp:405-407 */
    memcpy(rb, file, g); pos = g;
    int eof = g < cs;
    uint8_t last = rb[g - 1];
    if (search_chunk(&z, rb, g, &out)) goto fail;
    while (!eof) {                                      /* main.cpp:410-415 */
        rb[0] = last;
        g = n - pos < cs - 1 ? n - pos : cs - 1;
        memcpy(rb + 1, file + pos, g); pos += g;
        eof = g < cs - 1;
        last = g >= 1 ? rb[g - 1] : 0;                  /* rBuffer[gcount-1]; gcount==0 is UB, never used */
        if (search_chunk(&z, rb, g + 1, &out)) goto fail;
    }
    free(rb); free(z.pend);
    res->streams = out.v; res->n_streams = out.n;
    return 0;
fail:
    free(rb); free(z.pend); free(out.v);
    return -1;
}

/* ------------------------------------------------------------------------------------------ */
typedef struct { uint8_t c, w, m; } prm;
typedef struct { prm *v; int n, cap; } plist;
static void padd(plist *l, int c, int w, int m) {
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 128; l->v = (prm *)realloc(l->v, (size_t)l->cap * sizeof(prm)); }
    l->v[l->n].c = (uint8_t)c; l->v[l->n].w = (uint8_t)w; l->v[l->n].m = (uint8_t)m; l->n++;
}
/* testParamRange order: window desc, memlevel desc, clevel desc (main.cpp:739-745) */
static void prange(plist *l, int cmin, int cmax, int wmin, int wmax, int mmin, int mmax) {
    for (int w = wmax; w >= wmin; w--)
        for (int m = mmax; m >= mmin; m--)
            for (int c = cmax; c >= cmin; c--) padd(l, c, w, m);
}
/* tryParamsFastest/Fast/Default/Best, main.cpp:487-560 (each `return` on success == stop) */
static void phase_a(plist *l, int type) {
    int w = 10 + type / 4;
    switch (type % 4) {
    case 0: padd(l, 0, w, 8); padd(l, 1, w, 8); padd(l, 1, w, 9);
            prange(l, 1, 1, w, w, 1, 7); prange(l, 2, 9, w, w, 1, 9); break;
    case 1: prange(l, 2, 5, w, w, 8, 8); prange(l, 2, 5, w, w, 1, 7); prange(l, 2, 5, w, w, 9, 9);
            prange(l, 1, 1, w, w, 1, 9); prange(l, 6, 9, w, w, 1, 9); break;
    case 2: padd(l, 6, w, 8); padd(l, 6, w, 9); prange(l, 6, 6, w, w, 1, 7);
            prange(l, 1, 5, w, w, 1, 9); prange(l, 7, 9, w, w, 1, 9); break;
    default: prange(l, 7, 9, w, w, 8, 8); prange(l, 7, 9, w, w, 1, 7); prange(l, 7, 9, w, w, 9, 9);
             prange(l, 1, 6, w, w, 1, 9); break;
    }
}
/* brute-window continuation, main.cpp:590-601 */
static void phase_b(plist *l, int type) {
    int w = 10 + type / 4;
    if (w == 10) prange(l, 1, 9, 11, 15, 1, 9);
    else if (w == 15) prange(l, 1, 9, 10, 14, 1, 9);
    else { prange(l, 1, 9, 10, w - 1, 1, 9); prange(l, 1, 9, w + 1, 15, 1, 9); }
}

typedef struct { uint64_t *off; uint8_t *val; uint64_t n, cap; } dvec;

typedef struct {
    const uint8_t *orig, *infl; uint64_t cs, is;
    ora_stream_t *st;
    uint64_t *raw; uint8_t *rawv; uint64_t nraw;   /* current best diff list (raw positions) */
    uint64_t trials, bailed, hazard;
} sweep_ctx;

/* testDeflateParams, main.cpp:603-731 (one-shot bytes; shortcut = prefix) */
static int test_params(sweep_ctx *x, const ora_opts_t *o, prm p, uint8_t *buf, uint64_t cap) {
    uint64_t L; int fl = 0;
    x->trials++;
    if (ora_deflate(x->infl, x->is, p.c, p.w, p.m, buf, cap, &L, &fl) != 0) return -1;
    if (fl) x->hazard++;
    int full = 1, fullmatch = 0;
    if (x->cs > o->shortcut_len) {
        uint64_t k = L < o->shortcut_len ? L : o->shortcut_len, id = 0;
        for (uint64_t i = 0; i < k; i++) id += buf[i] == x->orig[i];
        if (id < (uint64_t)(o->shortcut_len - o->recomp_tresh)) full = 0;
    }
    if (!full) { x->bailed++; return 0; }
    int64_t d = (int64_t)(L - x->cs);
    uint64_t ad = (uint64_t)(d < 0 ? -d : d);
    if (ad > o->sizediff_tresh) return 0;
    uint64_t sm = L < x->cs ? L : x->cs, id = 0;
    for (uint64_t i = 0; i < sm; i++) id += buf[i] == x->orig[i];
    if (id > x->st->ident) {
        x->st->ident = id;
        x->st->clevel = p.c; x->st->window = p.w; x->st->memlevel = p.m;
        x->st->first_diff = -1;
        x->nraw = 0;
        if (id == x->cs) fullmatch = 1;
        else {
            if (id + o->mismatch_tol >= x->cs) fullmatch = 1;
            for (uint64_t i = 0; i < sm; i++)
                if (buf[i] != x->orig[i]) { x->raw[x->nraw] = i; x->rawv[x->nraw++] = x->orig[i]; }
            if (L < x->cs)
                for (uint64_t i = L; i < x->cs; i++) { x->raw[x->nraw] = i; x->rawv[x->nraw++] = x->orig[i]; }
            x->st->first_diff = (int64_t)x->raw[0];   /* deltaEncode main.cpp:757-763 */
        }
    }
    return fullmatch;
}

static int run_list(sweep_ctx *x, const ora_opts_t *o, const plist *l, uint8_t *buf, uint64_t cap) {
    for (int i = 0; i < l->n; i++) {
        int r = test_params(x, o, l->v[i], buf, cap);
        if (r < 0) return r;
        if (r) return 1;
    }
    return 0;
}

int ora_sweep(const uint8_t *file, uint64_t n, const ora_opts_t *o, ora_result_t *res) {
    dvec dv = {0};
    uint64_t trials = 0, bailed = 0, hazard = 0;
    for (uint64_t s = 0; s < res->n_streams; s++) {
        ora_stream_t *st = &res->streams[s];
        if (st->offset + st->comp_len > n) return -10;  /* reference reads past EOF -> garbage -> abort */
        const uint8_t *orig = file + st->offset;
        uint8_t *infl = (uint8_t *)malloc(st->infl_len ? st->infl_len : 1);
        uint64_t c, p;
        int r = ora_inflate(orig, st->comp_len, infl, st->infl_len, &c, &p);
        if (r != ORA_INF_END || p != st->infl_len) { free(infl); return -11; } /* main.cpp:450-452 abort() */
        uint64_t cap = ora_deflate_bound(st->infl_len, 15, 9) + 4096;
        uint64_t cap2 = ora_deflate_bound(st->infl_len, 10, 1) + 4096;
        if (cap2 > cap) cap = cap2;
        uint8_t *buf = (uint8_t *)malloc(cap);
        sweep_ctx x;
        memset(&x, 0, sizeof(x));
        x.orig = orig; x.infl = infl; x.cs = st->comp_len; x.is = st->infl_len; x.st = st;
        x.raw = (uint64_t *)malloc((st->comp_len + 1) * sizeof(uint64_t));
        x.rawv = (uint8_t *)malloc(st->comp_len + 1);
        plist a = {0};
        phase_a(&a, st->type);
        r = run_list(&x, o, &a, buf, cap);
        if (r >= 0 && (st->comp_len - st->ident) >= o->mismatch_tol && o->brute_window) {
            plist b = {0};
            phase_b(&b, st->type);
            r = run_list(&x, o, &b, buf, cap);
            free(b.v);
        }
        free(a.v);
        if (r < 0) { free(infl); free(buf); free(x.raw); free(x.rawv); return -12; }
        st->recomp = ((st->comp_len - st->ident) <= o->recomp_tresh) && st->ident > 0;
        st->n_trials = x.trials;
        trials += x.trials; bailed += x.bailed; hazard += x.hazard;
        /* keep the diff list only where it will be written (recomp streams) */
        st->diff_index = dv.n;
        st->n_diff = st->recomp ? x.nraw : 0;
        if (st->recomp && x.nraw) {
            if (dv.n + x.nraw > dv.cap) {
                dv.cap = (dv.n + x.nraw) * 2;
                dv.off = (uint64_t *)realloc(dv.off, dv.cap * sizeof(uint64_t));
                dv.val = (uint8_t *)realloc(dv.val, dv.cap);
            }
            for (uint64_t k = 0; k < x.nraw; k++) {
                dv.off[dv.n + k] = k == 0 ? 0 : x.raw[k] - x.raw[k - 1];
                dv.val[dv.n + k] = x.rawv[k];
            }
            dv.n += x.nraw;
        }
        free(infl); free(buf); free(x.raw); free(x.rawv);
    }
    res->diff_off = dv.off; res->diff_val = dv.val; res->n_diffs = dv.n;
    res->n_trials = trials; res->n_shortcut_bailed = bailed; res->n_hazard = hazard;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
typedef struct { uint8_t *b; uint64_t n, cap; } obuf;
static void ow(obuf *o, const void *p, uint64_t n) {
    if (o->n + n > o->cap) { o->cap = (o->n + n) * 2 + 64; o->b = (uint8_t *)realloc(o->b, o->cap); }
    memcpy(o->b + o->n, p, n); o->n += n;
}
static void ow8(obuf *o, uint64_t v) { ow(o, &v, 8); }
static void ow1(obuf *o, uint8_t v) { ow(o, &v, 1); }

int ora_write_atz(const uint8_t *file, uint64_t n, const ora_result_t *res, uint8_t **atz, uint64_t *atz_len) {
    obuf o = {0};
    uint64_t nrec = 0;
    for (uint64_t s = 0; s < res->n_streams; s++) nrec += res->streams[s].recomp;
    ow(&o, "ATZ\1", 4); ow8(&o, 0); ow8(&o, n); ow8(&o, nrec);
    for (uint64_t s = 0; s < res->n_streams; s++) {
        const ora_stream_t *st = &res->streams[s];
        if (!st->recomp) continue;
        ow8(&o, st->offset); ow8(&o, st->comp_len); ow8(&o, st->infl_len);
        ow1(&o, st->clevel); ow1(&o, st->window); ow1(&o, st->memlevel);
        ow8(&o, st->n_diff);
        if (st->n_diff) {
            ow8(&o, (uint64_t)st->first_diff);
            for (uint64_t k = 0; k < st->n_diff; k++) ow8(&o, res->diff_off[st->diff_index + k]);
            for (uint64_t k = 0; k < st->n_diff; k++) ow1(&o, res->diff_val[st->diff_index + k]);
        }
        uint8_t *infl = (uint8_t *)malloc(st->infl_len ? st->infl_len : 1);
        uint64_t c, p;
        ora_inflate(file + st->offset, st->comp_len, infl, st->infl_len, &c, &p);
        ow(&o, infl, st->infl_len);
        free(infl);
    }
    uint64_t lastos = 0, lastlen = 0;
    for (uint64_t s = 0; s < res->n_streams; s++) {
        const ora_stream_t *st = &res->streams[s];
        if (lastos + lastlen != st->offset) {
            if (st->offset < lastos + lastlen) { free(o.b); return -20; } /* uint64 wrap in copyto: UB */
            ow(&o, file + lastos + lastlen, st->offset - (lastos + lastlen));
        }
        if (!st->recomp) ow(&o, file + st->offset, st->comp_len);
        lastos = st->offset; lastlen = st->comp_len;
    }
    if (lastos + lastlen < n) ow(&o, file + lastos + lastlen, n - (lastos + lastlen));
    uint64_t total = o.n;
    memcpy(o.b + 4, &total, 8);
    *atz = o.b; *atz_len = o.n;
    return 0;
}

int ora_precompress(const uint8_t *file, uint64_t n, const ora_opts_t *o, uint8_t **atz,
                    uint64_t *atz_len, ora_result_t *res_out) {
    ora_result_t res;
    int r = ora_scan(file, n, o->chunksize, &res);
    if (r) return r;
    r = ora_sweep(file, n, o, &res);
    if (r == 0) r = ora_write_atz(file, n, &res, atz, atz_len);
    if (res_out) *res_out = res; else ora_result_free(&res);
    return r;
}

static uint64_t rd8(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

int ora_reconstruct(const uint8_t *atz, uint64_t n, uint8_t **out, uint64_t *out_len) {
    if (n < 28 || memcmp(atz, "ATZ\1", 4) != 0) return -2;    /* main.cpp:1018-1021 */
    if (rd8(atz + 4) != n) return -3;                         /* main.cpp:1022-1025 */
    uint64_t origlen = rd8(atz + 12), nstrms = rd8(atz + 20);
    obuf o = {0};
    if (nstrms == 0) {
        if (28 + origlen > n) return -4;
        ow(&o, atz + 28, origlen);
        *out = o.b; *out_len = o.n;
        return 0;
    }
    typedef struct { uint64_t off, cl, il, nd, fd, dpos, ipos; uint8_t c, w, m; } desc;
    desc *d = (desc *)calloc(nstrms, sizeof(desc));
    uint64_t lastos = 28;                                     /* readStreamdesc_ALL main.cpp:1031-1063 */
    for (uint64_t j = 0; j < nstrms; j++) {
        if (lastos + 35 > n) { free(d); return -4; }
        d[j].off = rd8(atz + lastos); d[j].cl = rd8(atz + lastos + 8); d[j].il = rd8(atz + lastos + 16);
        d[j].c = atz[lastos + 24]; d[j].w = atz[lastos + 25]; d[j].m = atz[lastos + 26];
        d[j].nd = rd8(atz + lastos + 27);
        if (d[j].nd) {
            d[j].fd = rd8(atz + lastos + 35);
            d[j].dpos = lastos + 43;
            d[j].ipos = 43 + d[j].nd * 9 + lastos;
            lastos = lastos + 43 + d[j].nd * 9 + d[j].il;
        } else {
            d[j].ipos = 35 + lastos;
            lastos = lastos + 35 + d[j].il;
        }
        if (lastos > n) { free(d); return -4; }
    }
    uint64_t residue = lastos, gapsum = 0, lo = 0, ll = 0;
    for (uint64_t j = 0; j < nstrms; j++) {
        if (lo + ll != d[j].off) {
            uint64_t g = d[j].off - (lo + ll);
            if (residue + gapsum + g > n) { free(d); free(o.b); return -5; }
            ow(&o, atz + residue + gapsum, g);
            gapsum += g;
        }
        uint64_t cap = d[j].cl + 65535, L;
        uint8_t *cb = (uint8_t *)calloc(cap + ora_deflate_bound(d[j].il, 10, 1), 1);
        int r = ora_deflate(atz + d[j].ipos, d[j].il, d[j].c, d[j].w, d[j].m, cb, cap, &L, NULL);
        if (r != 0) { free(cb); free(d); free(o.b); return -6; }   /* doDeflate abort() main.cpp:994-997 */
        if (d[j].nd) {
            uint64_t sum = 0;
            for (uint64_t i = 0; i < d[j].nd; i++) {
                uint64_t delta = rd8(atz + d[j].dpos + 8 * i);
                uint64_t at = d[j].fd + delta + sum;
                if (at < cap) cb[at] = atz[d[j].dpos + 8 * d[j].nd + i];
                sum += delta;
            }
        }
        ow(&o, cb, d[j].cl);
        free(cb);
        lo = d[j].off; ll = d[j].cl;
    }
    if (lo + ll < origlen) {
        uint64_t t = origlen - (lo + ll);
        if (residue + gapsum + t > n) { free(d); free(o.b); return -5; }
        ow(&o, atz + residue + gapsum, t);
    }
    free(d);
    *out = o.b; *out_len = o.n;
    return 0;
}

void ora_result_free(ora_result_t *res) {
    free(res->streams); free(res->diff_off); free(res->diff_val);
    memset(res, 0, sizeof(*res));
}
void ora_free(void *p) { free(p); }
