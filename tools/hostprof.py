"""Resolve an ATZ_HOSTPROF sample file (the last call's section): per function in libatz_accel (the
innermost inlined frame and the enclosing symbol, via llvm-symbolizer) and per other object.
usage: python3 tools/hostprof.py <file.prof> [top] [thread slots, e.g. 1,2,3]"""
import collections
import subprocess
import sys

LIB = "antiz_amd/_build/libatz_accel.so"


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    sections, cur = [], None
    for line in open(path):
        if line.startswith("#"):
            cur = []
            sections.append(cur)
            continue
        n, thr, obj, off, sym = line.split(None, 4)
        cur.append((int(n), obj, int(off, 16), sym.strip(), int(thr)))
    rows = sections[-1]
    total = sum(r[0] for r in rows)
    want = set(int(t) for t in sys.argv[3].split(",")) if len(sys.argv) > 3 else None   # thread slots (0: caller)
    if want is not None:
        rows = [r for r in rows if r[4] in want]
        total = sum(r[0] for r in rows)
    per_thr = collections.Counter()
    for r in rows:
        per_thr[(r[4], "libatz" if r[1].endswith("libatz_accel.so") else r[1].rsplit("/", 1)[-1])] += r[0]
    mine = [r for r in rows if r[1].endswith("libatz_accel.so")]
    other = collections.Counter()
    for n, obj, off, sym, _ in rows:
        if not obj.endswith("libatz_accel.so"):
            other[obj.rsplit("/", 1)[-1] + " " + sym] += n
    inner, outer, lines = collections.Counter(), collections.Counter(), collections.Counter()
    if mine:
        inp = "\n".join(hex(r[2]) for r in mine) + "\n"
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-symbolizer", "--obj=" + LIB, "--inlining", "--demangle"],
                             input=inp, capture_output=True, text=True).stdout.split("\n\n")
        for r, blk in zip(mine, out):
            ls = [x for x in blk.strip().split("\n") if x]
            fr = [(ls[i], ls[i + 1] if i + 1 < len(ls) else "") for i in range(0, len(ls), 2)]
            if not fr:
                continue
            inner[fr[0][0][:110]] += r[0]
            outer[fr[-1][0][:110]] += r[0]
            lines[fr[0][1].rsplit("/", 1)[-1]] += r[0]
    print("samples %d, in libatz_accel %d" % (total, sum(r[0] for r in mine)))
    for t in sorted(set(k[0] for k in per_thr)):
        print("thread %d: " % t + ", ".join("%s %d" % (k[1], v) for k, v in per_thr.most_common() if k[0] == t))
    for title, c in (("innermost function", inner), ("enclosing function", outer), ("source line", lines), ("other objects", other)):
        print("\n== %s" % title)
        for k, v in c.most_common(top):
            print("%6d %5.1f%%  %s" % (v, 100.0 * v / max(total, 1), k))


if __name__ == "__main__":
    main()
