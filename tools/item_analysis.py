import numpy as np, sys
z=np.load(sys.argv[1])
D=z['dur_all']; S=z['start_all']; ent=z['entries']; pcs=z['pieces']; rb=z['rb']; x=z['xcc']
w=ent>0
D=D[:,w]; S=S[:,w]; ent=ent[w]; pcs=pcs[w]; rb=rb[w]; x=x[w]
E=D+S
print('items',w.sum(),'iters',D.shape[0])
m=D.mean(0); sd=D.std(0)
print('dur mean over items %.2f, std across items of per-item mean %.3f, mean per-item std over iters %.3f'%(m.mean(), m.std(), sd.mean()))
print('start: mean %.2f p90 %.2f max %.2f'%(S.mean(), np.percentile(S.mean(0),90), S.max(1).mean()))
print('end (start+dur): p50 %.2f max per iter mean %.2f'%(np.median(E), E.max(1).mean()))
X=np.stack([np.ones_like(ent), ent, pcs],1).astype(float)
coef,res,_,_=np.linalg.lstsq(X,m,rcond=None)
pred=X@coef
print('fit dur = %.3f + %.5f*entries + %.5f*pieces ; R2 %.3f'%(coef[0],coef[1],coef[2], 1-((m-pred)**2).sum()/((m-m.mean())**2).sum()))
print('entries range', ent.min(), ent.max(), 'pieces range', pcs.min(), pcs.max())
for r in np.unique(rb): print(' rb',r,'n',(rb==r).sum(),'dur mean %.2f'%m[rb==r].mean(), 'ent mean %.0f pcs %.0f'%(ent[rb==r].mean(), pcs[rb==r].mean()))
for c in np.unique(x): print(' xcc',c,'dur mean %.2f'%m[x==c].mean(),'start %.2f'%S.mean(0)[x==c].mean())
# which item ends last per iteration: is it consistent?
last=E.argmax(1); print('last-ending item ids (top):', np.bincount(last).argsort()[-5:], np.sort(np.bincount(last))[-5:])
print('corr(per-item mean dur, start mean)=%.3f'%np.corrcoef(m, S.mean(0))[0,1])
