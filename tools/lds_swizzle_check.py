"""Enumerates LDS bank quads of the split cores' fragment reads
(gemm_s3.hip pswz) over gfx950's ds_read_b128 lane groups
(MI355X_MICROARCH.md, LDS): prints the worst n-way conflict of each read
pattern for the current and the previous BK = 32 swizzle, and checks that
ds_write_b128 staging stays conflict-free.  CPU only."""
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]


def cur(r, s):
    return s ^ ((((r >> 3) & 1) << 1) | ((r >> 4) & 1))


def prev(r, s):
    return s ^ ((r >> 2) & 3)


def worst_read(f, rowfn, slotfn):
    w = 0
    for base in range(0, 256, 32):
        for g in GROUPS:
            cnt = {}
            for lane in g:
                r = base + rowfn(lane)
                q = (r * 4 + f(r, slotfn(lane))) % 16  # 64-B rows: 4 quads each
                cnt[q] = cnt.get(q, 0) + 1
            w = max(w, max(cnt.values()))
    return w


def worst_write(f):
    w = 0
    for base in range(0, 256, 16):
        for g0 in range(0, 64, 8):
            cnt = {}
            for lane in range(g0, g0 + 8):
                r, s = base + lane // 4, lane % 4
                q = (r * 4 + f(r, s)) % 8  # ds_write_b128: banks (a/4) mod 32
                cnt[q] = cnt.get(q, 0) + 1
            w = max(w, max(cnt.values()))
    return w


if __name__ == "__main__":
    pats = {"16x16x32 (row l&15 (+16h), slot l>>4)": (lambda l: l & 15, lambda l: l >> 4),
            "16x16x32 h=1": (lambda l: 16 + (l & 15), lambda l: l >> 4),
            "32x32x16 step 0": (lambda l: l & 31, lambda l: l >> 5),
            "32x32x16 step 1": (lambda l: l & 31, lambda l: 2 + (l >> 5))}
    for name, (rf, sf) in pats.items():
        print(f"{name}: current {worst_read(cur, rf, sf)}-way, previous {worst_read(prev, rf, sf)}-way")
    print(f"ds_write_b128 staging: current {worst_write(cur)}-way, previous {worst_write(prev)}-way")
    for r in range(256):
        assert sorted(cur(r, s) for s in range(4)) == [0, 1, 2, 3]
