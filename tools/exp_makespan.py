"""Dev: does queue order shrink the drain tail? A lane-level model of the persistent queue
(2048 waves x 64 lanes pull rays in queue order; a ray costs its attempt count) on the
per-ray costs of the flat 1e6 batch (gpurun_out/cost1e6.npz from tools/exp_cost.py), for the
sampler's order, true longest-first (LPT), simple start-point scores, and a gradient-boosted
predictor of log(attempts) from 12 start-point features (/tmp/pred.npy)."""
import numpy as np, heapq
z=np.load('/root/repo/gpurun_out/cost1e6.npz')
att=z['att'].astype(np.int64); n=len(att)
LANES=2048*64
def makespan(order, lanes=LANES):
    # lanes pull rays in queue order; each ray costs att iterations (unit time)
    a=att[order]
    h=[0]*lanes  # finish times
    # first 'lanes' rays start at 0
    fin=np.zeros(lanes,dtype=np.int64)
    m=min(lanes,n)
    fin[:m]=a[:m]
    h=list(zip(fin.tolist(),range(lanes)))
    heapq.heapify(h)
    for i in range(m,n):
        t,l=heapq.heappop(h)
        heapq.heappush(h,(t+int(a[i]),l))
    ts=[t for t,_ in h]
    return max(ts), np.mean(ts)
tot=att.sum()/LANES
print('ideal (total/lanes)', tot)
print('given order', makespan(np.arange(n)))
print('LPT (true cost desc)', makespan(np.argsort(-att,kind='stable')))
x=z['x0'].astype(np.float64); k=z['k0'].astype(np.float64)
r=np.linalg.norm(x,axis=0); kn=k/np.linalg.norm(k,axis=0); kr=np.sum(kn*x,axis=0)/r
ct=x[2]/r
for name,score in [('-k_r',-kr),('1/r',1/r),('-k_r/r', -kr/r), ('-k_r - r/20',-kr-r/20)]:
    o=np.argsort(-score,kind='stable')
    print(name, makespan(o), 'corr', np.corrcoef(np.argsort(np.argsort(score)),np.argsort(np.argsort(att)))[0,1])
pred=np.load('/tmp/pred.npy')
print('GBM pred', makespan(np.argsort(-pred,kind='stable')))
rng=np.random.default_rng(1)
for q in [0.01,0.03,0.1,0.3]:
    o=np.argsort(-pred,kind='stable'); m=int(q*n)
    head=o[:m]; rest=o[m:].copy(); rng.shuffle(rest)
    print('top',q, makespan(np.concatenate([head,rest])))
# true-cost top q then random (upper bound of this strategy)
for q in [0.01,0.03]:
    o=np.argsort(-att,kind='stable'); m=int(q*n); head=o[:m]; rest=o[m:].copy(); rng.shuffle(rest)
    print('true top',q, makespan(np.concatenate([head,rest])))
