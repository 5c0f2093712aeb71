/*
 * ora_inflate.c -- plain-C restatement of zlib 1.2.8 inflate as the AntiZ scanner observes it
 * (TEST INFRASTRUCTURE ONLY).
 *
 * What the reference's scanner (main.cpp:205-246 via ZlibWrapper.h:58-82) reads back from zlib is:
 * the return class (Z_STREAM_END / error / ran out of input), total_in, total_out and avail_in.
 * zlib 1.2.8 (Z/inflate.c:605-1252, Z/inffast.c:67-340, Z/inftrees.c:32-306) pulls input bytes
 * only as NEEDBITS/PULLBYTE require them and (inflate_fast) hands whole unused bytes back, so:
 *   - Z_STREAM_END   : total_in = exact stream length (trailer included, Z/inflate.c:1174-1195)
 *   - error          : total_in = ceil(bits required up to the failing item / 8)
 *   - out of input   : total_in = everything offered (avail_in == 0)
 * This decoder tracks `need` = the highest bit position zlib would have required; every read
 * beyond the offered bytes returns ORA_INF_NEED_INPUT first, as NEEDBITS does.
 * Table quirks restated: an empty code-length code decodes every length as 0 with 1 bit
 * (Z/inftrees.c:116-127 + Z/inflate.c:969-974 ignore `op`); incomplete lit/len or distance
 * codes are accepted only when the longest code has 1 bit, and an unused 1-bit pattern /
 * an empty distance code fails after 1 bit (Z/inftrees.c:139-141, 293-303); fixed codes 286/287
 * and distance 30/31 are invalid after their full 8/5 bits (lext/dext sentinels).
 */
#include "atz_oracle.h"
#include <stdlib.h>
#include <string.h>

uint32_t ora_adler32(uint32_t adler, const uint8_t *buf, uint64_t len) { /* Z/adler32.c:65 */
    uint32_t a = adler & 0xffff, b = adler >> 16;
    while (len) {
        uint64_t k = len < 5552 ? len : 5552;
        len -= k;
        while (k--) { a += *buf++; b += a; }
        a %= 65521; b %= 65521;
    }
    return (b << 16) | a;
}

typedef struct {
    const uint8_t *in; uint64_t n;
    uint64_t pos;   /* bits consumed (dropped) */
    uint64_t need;  /* highest bit position required so far */
    uint8_t *out; uint64_t out_len, out_cap; int own;
} IS;

#define NEED_INPUT -2
#define BAD -1

static int need_bits(IS *s, unsigned k) {
    uint64_t p = s->pos + k;
    if (p > s->need) s->need = p;
    return p <= 8 * s->n ? 0 : NEED_INPUT;
}
static unsigned peek(IS *s, unsigned k) {  /* bits beyond the input read as zero */
    unsigned v = 0;
    for (unsigned i = 0; i < k; i++) {
        uint64_t b = s->pos + i;
        if (b < 8 * s->n) v |= (unsigned)((s->in[b >> 3] >> (b & 7)) & 1) << i;
    }
    return v;
}
static int getbits(IS *s, unsigned k, unsigned *v) {
    int r = need_bits(s, k);
    if (r) return r;
    *v = peek(s, k);
    s->pos += k;
    return 0;
}
static int emit(IS *s, uint8_t b) {
    if (s->out_len >= s->out_cap) {
        if (!s->own) return BAD;           /* caller buffer full: treat as error (not used by scanner) */
        uint64_t nc = s->out_cap ? s->out_cap * 2 : 65536;
        uint8_t *p = (uint8_t *)realloc(s->out, nc);
        if (!p) return BAD;
        s->out = p; s->out_cap = nc;
    }
    s->out[s->out_len++] = b;
    return 0;
}

typedef struct {
    uint16_t count[16];
    uint16_t sym[320];
    int max;        /* longest code length present (0: none) */
    int incomplete; /* allowed-incomplete (max==1) or empty */
} Huff;

/* inflate_table acceptance (Z/inftrees.c:32-141); type 0 CODES, 1 LENS, 2 DISTS.  0 ok, -1 bad */
static int build(Huff *h, const uint16_t *lens, int n, int type) {
    memset(h->count, 0, sizeof(h->count));
    for (int i = 0; i < n; i++) h->count[lens[i]]++;
    int max;
    for (max = 15; max >= 1; max--) if (h->count[max]) break;
    h->max = max;
    h->incomplete = 0;
    if (max == 0) { h->incomplete = 1; return 0; }
    int left = 1;
    for (int l = 1; l <= 15; l++) { left <<= 1; left -= h->count[l]; if (left < 0) return -1; }
    if (left > 0 && (type == 0 || max != 1)) return -1;
    if (left > 0) h->incomplete = 1;
    uint16_t offs[16]; offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = (uint16_t)(offs[l] + h->count[l]);
    for (int i = 0; i < n; i++) if (lens[i]) h->sym[offs[lens[i]]++] = (uint16_t)i;
    return 0;
}

/* returns symbol >=0, or BAD (invalid code; need already accounts its bits), or NEED_INPUT */
static int decode(IS *s, const Huff *h, int cl_quirk) {
    if (h->max == 0) {
        /* empty table: 1-bit invalid entries (Z/inftrees.c:116-127) */
        int r = need_bits(s, 1); if (r) return r;
        s->pos += 1;
        return cl_quirk ? 0 : BAD;
    }
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; len++) {
        uint64_t b = s->pos + len - 1;
        if (b >= 8 * s->n) { need_bits(s, (unsigned)len); return NEED_INPUT; }
        code |= (s->in[b >> 3] >> (b & 7)) & 1;
        int count = h->count[len];
        if (code - count < first) {
            need_bits(s, (unsigned)len);
            s->pos += len;
            return h->sym[index + (code - first)];
        }
        index += count; first += count; first <<= 1; code <<= 1;
        if (h->incomplete && len == 1) {       /* the unused 1-bit pattern */
            need_bits(s, 1); s->pos += 1;
            return BAD;
        }
    }
    return BAD;  /* unreachable for accepted codes */
}

static const uint16_t LBASE[29] = {3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258};
static const uint16_t LEXT[29] = {0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0};
static const uint16_t DBASE[30] = {1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577};
static const uint16_t DEXT[30] = {0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13};
static const uint8_t CLORDER[19] = {16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15};

#define TRY(x) do { int r_ = (x); if (r_) return r_; } while (0)

static int codes(IS *s, const Huff *lh, const Huff *dh) {
    for (;;) {
        int sym = decode(s, lh, 0);
        if (sym < 0) return sym;
        if (sym < 256) { TRY(emit(s, (uint8_t)sym)); continue; }
        if (sym == 256) return 0;
        sym -= 257;
        if (sym >= 29) return BAD;                 /* fixed 286/287 */
        unsigned e;
        TRY(getbits(s, LEXT[sym], &e));
        unsigned len = LBASE[sym] + e;
        int ds = decode(s, dh, 0);
        if (ds < 0) return ds;
        if (ds >= 30) return BAD;                  /* fixed 30/31 */
        TRY(getbits(s, DEXT[ds], &e));
        uint64_t dist = DBASE[ds] + e;
        if (dist > s->out_len) return BAD;         /* invalid distance too far back */
        for (unsigned i = 0; i < len; i++) TRY(emit(s, s->out[s->out_len - dist]));
    }
}

static int body(IS *s) {
    unsigned v;
    /* HEAD, Z/inflate.c:640-685 (wrap=1, wbits=15 from inflateInit) */
    TRY(need_bits(s, 16));
    unsigned cmf = peek(s, 8);
    s->pos += 8;
    unsigned flg = peek(s, 8);
    s->pos -= 8;
    if (((cmf << 8) + flg) % 31) return BAD;
    if ((cmf & 15) != 8) return BAD;
    if ((cmf >> 4) + 8 > 15) return BAD;
    s->pos += 16;
    if (flg & 0x20) { TRY(need_bits(s, 32)); return BAD; /* Z_NEED_DICT: not a stream end */ }
    int last;
    do {
        TRY(getbits(s, 1, &v)); last = (int)v;
        TRY(need_bits(s, 2));
        v = peek(s, 2); s->pos += 2;
        if (v == 0) {                               /* STORED */
            s->pos = (s->pos + 7) & ~7ull;
            TRY(need_bits(s, 32));
            unsigned len = peek(s, 16);
            s->pos += 16;
            unsigned nlen = peek(s, 16);
            s->pos += 16;
            if (len != (~nlen & 0xffff)) return BAD;
            for (unsigned i = 0; i < len; i++) {
                TRY(need_bits(s, 8));
                TRY(emit(s, s->in[s->pos >> 3]));
                s->pos += 8;
            }
        } else if (v == 1) {                        /* FIXED */
            static Huff fl, fd; static int fi = 0;
            if (!fi) {
                uint16_t l[320]; int i;
                for (i = 0; i < 144; i++) l[i] = 8;
                for (; i < 256; i++) l[i] = 9;
                for (; i < 280; i++) l[i] = 7;
                for (; i < 288; i++) l[i] = 8;
                build(&fl, l, 288, 1);
                for (i = 0; i < 32; i++) l[i] = 5;
                build(&fd, l, 32, 2);
                fi = 1;
            }
            TRY(codes(s, &fl, &fd));
        } else if (v == 2) {                        /* DYNAMIC, Z/inflate.c:908-1013 */
            unsigned nlen, ndist, ncode;
            TRY(need_bits(s, 14));
            nlen = peek(s, 5) + 257; s->pos += 5;
            ndist = peek(s, 5) + 1; s->pos += 5;
            ncode = peek(s, 4) + 4; s->pos += 4;
            if (nlen > 286 || ndist > 30) return BAD;
            uint16_t lens[320];
            memset(lens, 0, sizeof(lens));
            for (unsigned i = 0; i < ncode; i++) { TRY(getbits(s, 3, &v)); lens[CLORDER[i]] = (uint16_t)v; }
            Huff ch;
            if (build(&ch, lens, 19, 0)) return BAD;
            unsigned have = 0;
            uint16_t ll[320];
            while (have < nlen + ndist) {
                int sym = decode(s, &ch, 1);
                if (sym < 0) return sym;
                if (sym < 16) { ll[have++] = (uint16_t)sym; continue; }
                /* the repeat code's bits were dropped by decode(); zlib needs them + extra first */
                unsigned copy, len = 0;
                if (sym == 16) {
                    TRY(need_bits(s, 2));
                    if (have == 0) return BAD;
                    len = ll[have - 1];
                    copy = 3 + peek(s, 2); s->pos += 2;
                } else if (sym == 17) {
                    TRY(need_bits(s, 3));
                    copy = 3 + peek(s, 3); s->pos += 3;
                } else {
                    TRY(need_bits(s, 7));
                    copy = 11 + peek(s, 7); s->pos += 7;
                }
                if (have + copy > nlen + ndist) return BAD;
                while (copy--) ll[have++] = (uint16_t)len;
            }
            if (ll[256] == 0) return BAD;
            Huff lh, dh;
            if (build(&lh, ll, (int)nlen, 1)) return BAD;
            if (build(&dh, ll + nlen, (int)ndist, 2)) return BAD;
            TRY(codes(s, &lh, &dh));
        } else {
            return BAD;                              /* invalid block type */
        }
    } while (!last);
    /* CHECK, Z/inflate.c:1174-1195 */
    s->pos = (s->pos + 7) & ~7ull;
    TRY(need_bits(s, 32));
    uint32_t want = 0;
    for (int i = 0; i < 4; i++) { want = (want << 8) | s->in[(s->pos >> 3) + i]; }
    s->pos += 32;
    if (want != ora_adler32(1, s->out, s->out_len)) return BAD;
    return 0;
}

int ora_inflate(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                uint64_t *consumed, uint64_t *produced) {
    IS s;
    memset(&s, 0, sizeof(s));
    s.in = in; s.n = n;
    if (out) { s.out = out; s.out_cap = out_cap; s.own = 0; }
    else { s.own = 1; }
    int r = body(&s);
    int st;
    if (r == 0) { st = ORA_INF_END; *consumed = s.pos >> 3; }
    else if (r == NEED_INPUT) { st = ORA_INF_NEED_INPUT; *consumed = n; }
    else { st = ORA_INF_ERROR; uint64_t c = (s.need + 7) >> 3; *consumed = c > n ? n : c; }
    *produced = s.out_len;
    if (s.own) free(s.out);
    return st;
}
