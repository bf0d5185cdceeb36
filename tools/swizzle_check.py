#!/usr/bin/env python3
"""Exhaustive LDS bank check of igemm_x9.h pl_off (bf16 planes, 64-B rows, 16-B chunks)
for the three access patterns that use it (MI355X_MICROARCH.md §LDS lane groups):
  * ds_read_b128 fragment reads: 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}
    (and +32), lane -> row = base + (lane & 15), chunk = lane >> 4;
  * split-at-staging non-KC writes (ds_write_b128, 8 contiguous lanes): rows 4t + q
    of 8 consecutive t, one chunk;
  * KC writes: 8 lanes = 2 rows x 4 chunks.
A 16-B access's bank slot is (byte address / 16) mod 16.  Prints the worst
multiplicity per pattern (1 = conflict-free).   python tools/swizzle_check.py"""


def pl_off(row, q):   # bf16 elements, as igemm_x9.h
    h4 = 0x1320
    return (row ^ ((row >> 4) & 1)) * 32 + 8 * (q ^ ((h4 >> (4 * ((row >> 2) & 3))) & 3))


def slot(row, q):
    return (2 * pl_off(row, q) // 16) % 16


READ = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
READ += [[x + 32 for x in g] for g in READ]


def worst(groups):
    return max(max(g.count(x) for x in g) for g in groups)


reads = [[slot(base + (l & 15), l >> 4) for l in g] for base in range(0, 256, 16) for g in READ]
nonkc = [[slot(4 * (t0 + t) + q, c) for t in range(8)] for t0 in range(0, 64, 8) for c in range(4) for q in range(4)]
kc = [[slot(r0 + i // 4, i % 4) for i in range(8)] for r0 in range(0, 256, 2)]
print("reads", worst(reads), "non-KC writes", worst(nonkc), "KC writes", worst(kc))
assert worst(reads) == worst(nonkc) == worst(kc) == 1
