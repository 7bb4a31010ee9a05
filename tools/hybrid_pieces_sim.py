# Column-run pieces (cap 16 entries) of a HYBRID layout for the reddit-like stand-in, computed
# from the pattern (no GPU): every stored entry runs either in a row block (A rows staged in LDS,
# the entry's B row gathered, as k_sddmm_rb does today) or in a column block (B rows staged, the
# entry's A row gathered: the same kernel on the transposed pattern S^T with A and B swapped,
# writing the same CSR positions). An entry moves to the column block when its run there is
# longer than its run in the row block. Rows and columns are both in degree-sorted order.
#     python3 tools/hybrid_pieces_sim.py <scale> <RB> [iterations]
import sys
import time

import numpy as np

sys.path.insert(0, 'sddmm-gpu_amd')
from bsmr import synth  # noqa: E402

scale = float(sys.argv[1])
RB = int(sys.argv[2])
ITERS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
PMAX = 16
t = time.time()
M, N, rp, ci = synth.reddit_like(scale)
rp = np.asarray(rp, dtype=np.int64)
ci = np.asarray(ci, dtype=np.int64)
rdeg = np.diff(rp)
rows = np.repeat(np.arange(M), rdeg)
cdeg = np.bincount(ci, minlength=N)
nnz = len(ci)
print('gen', round(time.time() - t, 1), 's  M', M, 'N', N, 'nnz', nnz, flush=True)


def rank_of(deg):
    order = np.argsort(-deg, kind='stable')
    pos = np.empty(len(deg), np.int64)
    pos[order] = np.arange(len(deg))
    return pos


rpos, cpos = rank_of(rdeg), rank_of(cdeg)
key_r = (rpos[rows] // RB) * N + ci          # row block x column: one B-row gather per piece
key_c = (cpos[ci] // RB) * M + rows          # column block x row: one A-row gather per piece


def group_counts(key, mask):
    """(run length each entry would have in its group of this mode: the mode's current members
    plus the entry itself if it is not one, pieces of the members, groups of the members)"""
    u, cnt = np.unique(key[mask], return_counts=True)
    i = np.minimum(np.searchsorted(u, key), max(len(u) - 1, 0))
    hit = (u[i] == key) if len(u) else np.zeros(nnz, bool)
    run = np.where(hit, cnt[i] if len(u) else 0, 0) + (~mask)
    return run, int(((cnt + PMAX - 1) // PMAX).sum()), len(cnt)


def blocks(key_blk, mask):
    return len(np.unique(key_blk[mask]))


allm = np.ones(nnz, bool)
cr, pr, _ = group_counts(key_r, allm)
print(f'row blocks only        pieces {pr:,}  entries/piece {nnz / pr:.2f}  '
      f'B-row bytes {pr * 512 / 1e9:.2f} GB (K=128 fp32)', flush=True)
col = np.zeros(nnz, bool)
cc, pc0, _ = group_counts(key_c, allm)  # first decision: each side with every entry
print(f"column blocks only     pieces {pc0:,}  entries/piece {nnz / pc0:.2f}", flush=True)
for it in range(ITERS):
    new = cc > cr
    if np.array_equal(new, col):
        break
    col = new
    cr, pr, _ = group_counts(key_r, ~col)
    cc, pc, _ = group_counts(key_c, col)
    nrb = blocks(rpos[rows] // RB, ~col)
    ncb = blocks(cpos[ci] // RB, col)
    print(f'hybrid iter {it}: row-mode entries {int((~col).sum()):,} pieces {pr:,}; '
          f'column-mode entries {int(col.sum()):,} pieces {pc:,}; total pieces {pr + pc:,} '
          f'({nnz / (pr + pc):.2f} entries/piece, gathers {(pr + pc) * 512 / 1e9:.2f} GB); '
          f'row blocks {nrb}, column blocks {ncb}', flush=True)
