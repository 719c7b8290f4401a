import sys, os, time
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import numpy as np, synth
from simple_pbft_amd import Verifier
from simple_pbft_amd.pbftv import verify_msg_batch
ver = Verifier()
pub, reqs, votes, vsig, replies, rsig, checks = synth.config1_cluster(1000)
ver.register_keys(pub)
node_of = {nid: j for j, nid in enumerate(synth.NODES)}
vk = np.array([node_of[v[3]] for v in votes], np.uint32)
rk = np.array([node_of[r[3]] for r in replies], np.uint32)
vi = np.array([c[1] for c in checks if c[0] == "vote"], np.int64)
ri = np.array([c[1] for c in checks if c[0] == "reply"], np.int64)
seq_to_r = {reqs[r][3]: r for r in range(1000)}
groups = {}
for j in vi: groups.setdefault(seq_to_r[votes[j][1]], []).append(votes[j])
def t(f, n=5):
    f(); ts=[]
    for _ in range(n):
        a=time.perf_counter(); f(); ts.append(time.perf_counter()-a)
    return min(ts)*1e3
r = {}
r['digest_request'] = t(lambda: ver.digest_request_batch(reqs))
r['digest_vote'] = t(lambda: ver.digest_vote_batch(votes))
r['digest_reply'] = t(lambda: ver.digest_reply_batch(replies))
vd = ver.digest_vote_batch(votes); rd = ver.digest_reply_batch(replies); req_d = ver.digest_request_batch(reqs)
H = np.concatenate([vd[vi], rd[ri]]); S = np.concatenate([vsig[vi], rsig[ri]]); K = np.concatenate([vk[vi], rk[ri]])
r['gather'] = t(lambda: (np.concatenate([vd[vi], rd[ri]]), np.concatenate([vsig[vi], rsig[ri]]), np.concatenate([vk[vi], rk[ri]])))
r['verify_batch'] = t(lambda: ver.verify_batch(H, S, K))
def vm():
    for rr, vv in groups.items():
        verify_msg_batch(synth.VIEW, -1, req_d[rr].tobytes(), [v[0] for v in vv], [v[1] for v in vv], [v[2] for v in vv])
r['verify_msg_loop'] = t(vm)
print(r)
