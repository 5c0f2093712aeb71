/* zref_shim.c -- thin C entry points onto the REFERENCE's own vendored zlib 1.2.8 (oracle/_ref/libz128.a),
 * compiled by build_ref.sh into oracle/_ref/libzref.so.  Test infrastructure only: it lets tests
 * pin the plain-C restatement (ora_*.c) and the HIP product against zlib 1.2.8 itself, calling it
 * exactly the way main.cpp does. */
#include <string.h>
#include <stdlib.h>
#include "zlib.h"

/* one deflate(Z_FINISH) with unlimited output (testDeflateParams' bytes, main.cpp:616-666) */
int zref_deflate(const unsigned char *in, unsigned long n, int c, int w, int m,
                 unsigned char *out, unsigned long cap, unsigned long *len) {
    z_stream s; memset(&s, 0, sizeof(s));
    if (deflateInit2(&s, c, Z_DEFLATED, w, m, Z_DEFAULT_STRATEGY) != Z_OK) return -100;
    s.next_in = (Bytef *)in; s.avail_in = (uInt)n; s.next_out = out; s.avail_out = (uInt)cap;
    int r = deflate(&s, Z_FINISH);
    *len = s.total_out;
    deflateEnd(&s);
    return r == Z_STREAM_END ? 0 : r;
}

unsigned long zref_deflate_bound(unsigned long n, int c, int w, int m) {
    z_stream s; memset(&s, 0, sizeof(s));
    if (deflateInit2(&s, c, Z_DEFLATED, w, m, Z_DEFAULT_STRATEGY) != Z_OK) return 0;
    unsigned long b = deflateBound(&s, n);
    deflateEnd(&s);
    return b;
}

/* the reference's two-call shortcut sequence, main.cpp:627-666: returns total_out after each call */
int zref_deflate_shortcut(const unsigned char *in, unsigned long n, int c, int w, int m, unsigned sl,
                          unsigned char *out, unsigned long *len1, unsigned long *len2) {
    z_stream s; memset(&s, 0, sizeof(s));
    if (deflateInit2(&s, c, Z_DEFLATED, w, m, Z_DEFAULT_STRATEGY) != Z_OK) return -100;
    unsigned long bound = deflateBound(&s, n);
    s.next_in = (Bytef *)in; s.avail_in = (uInt)n; s.next_out = out; s.avail_out = sl;
    int r = deflate(&s, Z_FINISH);
    *len1 = s.total_out;
    if (r != Z_OK && r != Z_STREAM_END) { deflateEnd(&s); return -101; }
    s.avail_out = (uInt)(bound - sl);
    r = deflate(&s, Z_FINISH);
    *len2 = s.total_out;
    deflateEnd(&s);
    return r == Z_STREAM_END ? 0 : r;
}

/* ZlibInflator usage by the scanner (ZlibWrapper.h:58-75, main.cpp:228-239): inflateReset +
 * inflate(Z_SYNC_FLUSH) into a `bufsz` buffer, then continuePrev while avail_out == 0. */
int zref_inflate_scan(const unsigned char *in, unsigned long n, unsigned long bufsz,
                      int *ret_first, unsigned long *tin_first, int *ret_last,
                      unsigned long *tin, unsigned long *tout, unsigned long *avail_in) {
    z_stream s; memset(&s, 0, sizeof(s));
    if (inflateInit(&s) != Z_OK) return -100;
    unsigned char *ob = (unsigned char *)malloc(bufsz);
    s.next_in = (Bytef *)in; s.avail_in = (uInt)n; s.next_out = ob; s.avail_out = (uInt)bufsz;
    int r = inflate(&s, Z_SYNC_FLUSH);
    *ret_first = r; *tin_first = s.total_in;
    while (s.avail_out == 0) { s.next_out = ob; s.avail_out = (uInt)bufsz; r = inflate(&s, Z_SYNC_FLUSH); }
    *ret_last = r; *tin = s.total_in; *tout = s.total_out; *avail_in = s.avail_in;
    inflateEnd(&s); free(ob);
    return 0;
}

/* doInflate (main.cpp:461-486): one-shot Z_FINISH into exactly `cap` bytes */
int zref_inflate(const unsigned char *in, unsigned long n, unsigned char *out, unsigned long cap,
                 unsigned long *tin, unsigned long *tout) {
    z_stream s; memset(&s, 0, sizeof(s));
    s.next_in = (Bytef *)in; s.avail_in = (uInt)n;
    if (inflateInit(&s) != Z_OK) return -100;
    s.next_out = out; s.avail_out = (uInt)cap;
    int r = inflate(&s, Z_FINISH);
    *tin = s.total_in; *tout = s.total_out;
    inflateEnd(&s);
    return r;
}
