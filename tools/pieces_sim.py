# Column-run pieces of the row-block layout (cap 16 entries) for two launch row orders of the
# reddit-like stand-in, computed from the pattern (no GPU): python3 tools/pieces_sim.py <scale> <RB>
import sys, time, numpy as np
sys.path.insert(0, 'sddmm-gpu_amd')
from bsmr import synth
scale = float(sys.argv[1]); RB = int(sys.argv[2])
t = time.time()
M, N, rp, ci = synth.reddit_like(scale)
rp = np.asarray(rp, dtype=np.int64); ci = np.asarray(ci, dtype=np.int64)
deg = np.diff(rp)
rows = np.repeat(np.arange(M), deg)
print('gen', round(time.time() - t, 1), 's  M', M, 'nnz', len(ci), flush=True)
def pieces(pos, pmax=16):
    key = (pos[rows] // RB) * N + ci
    _, cnt = np.unique(key, return_counts=True)
    return int(((cnt + pmax - 1) // pmax).sum()), len(cnt)
ident = np.arange(M)
order = np.argsort(-deg, kind='stable'); pos_deg = np.empty(M, np.int64); pos_deg[order] = np.arange(M)
for name, pos in [('original (random ids)', ident), ('degree-sorted', pos_deg)]:
    p, d = pieces(pos)
    print(f'{name:24s} pieces {p:,}  distinct (block,col) {d:,}  entries/piece {len(ci)/p:.2f}', flush=True)
