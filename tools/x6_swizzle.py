"""Exhaustive search for the LDS chunk swizzle of ocppo_gemm.hip (x6_chunk_off): plane rows in
128-B pairs, 16-B chunk index XOR H(row), H = G[(row / 4) % 8] for a bijection G of 0..7, such that
ds_read_b128 fragment reads (MI355X_MICROARCH.md's four 16-lane groups, 64 banks) and the
ds_write_b64 stash writes (16-lane groups, 32 banks) of both operand orientations are conflict
free. Prints the number of solutions and the first few; the kernel uses G = bit reversal.
"""
import itertools
G_READ = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
          list(range(4,12))+list(range(16,20))+list(range(28,32)),
          list(range(32,36))+list(range(44,48))+list(range(52,60)),
          list(range(36,44))+list(range(48,52))+list(range(60,64))]
def addr(row, c, G):
    H = G[(row >> 2) & 7]
    return (row >> 1) * 128 + 16 * ((((row & 1) << 2) | c) ^ H)
def reads_ok(G):
    for base in (0, 16, 32, 48):
        for grp in G_READ:
            slots = set()
            for l in grp:
                a = addr(base + (l & 15), l >> 4, G)
                slots.add((a // 16) % 16)
            if len(slots) != 16: return False
    return True
def kc_writes_ok(G, ROWS=128):
    # piece p: kq = p & 7, rq = p >> 3; row = 4rq + j; k = 4kq -> chunk kq>>1, half kq&1
    for j in range(4):
        for g0 in range(0, 256, 16):
            slots = set()
            for p in range(g0, g0 + 16):
                kq, rq = p & 7, p >> 3
                if rq * 4 >= ROWS: break
                row = 4 * rq + j
                a = addr(row, kq >> 1, G) + (kq & 1) * 8
                slots.add((a // 8) % 16)
            if slots and len(slots) != 16: return False
    return True
def mc_writes_ok(G, ROWS=128):
    # new mapping: 16 lanes = 8 row quads x 2 k quads
    nrq = ROWS // 4
    for j in range(4):
        for g0 in range(0, 256, 16):
            slots = set()
            for p in range(g0, g0 + 16):
                rq = (p & 7) + 8 * ((p >> 4) % (nrq // 8))
                kq = ((p >> 3) & 1) + 2 * ((p >> 4) // (nrq // 8))
                if kq >= 8: break
                row = 4 * rq + j
                a = addr(row, kq >> 1, G) + (kq & 1) * 8
                slots.add((a // 8) % 16)
            if slots and len(slots) != 16: return False
    return True
sols = []
for G in itertools.permutations(range(8)):
    if reads_ok(G) and kc_writes_ok(G) and mc_writes_ok(G) and kc_writes_ok(G, 64) and mc_writes_ok(G, 64):
        sols.append(G)
print(len(sols), sols[:5])
