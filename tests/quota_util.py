"""Shared setup for the quota-gated scheduling tests (CPU: oracle as the engine; GPU: libgpuscore)."""
import numpy as np

from koordinator_amd import config, synth
from koordinator_amd.quota import ElasticQuotaPlugin

RES = ("cpu", "memory")


def setup(nodes=1000, pods=300, seed=0):
    c = synth.make_cluster(nodes, pods, seed)
    c.pods["requests"][::11, 0] = 1_000_000      # 1000-core pods: no feasible node (exercises the unreserve repair)
    c.pods["request_mask"][::11] |= 0x1
    cfg = config.make_config(c.num_nodes)
    return c, cfg


def plugin(lib=None, check_parent=True):
    p = ElasticQuotaPlugin(resources=RES, enable_check_parent_quota=check_parent, lib=lib)
    p.update_cluster_total_resource({"cpu": 400_000, "memory": 800 << 30})
    p.on_quota_add("team-a", max={"cpu": 250_000, "memory": 600 << 30}, min={"cpu": 100_000, "memory": 200 << 30})
    p.on_quota_add("team-a-1", parent="team-a", max={"cpu": 150_000, "memory": 400 << 30},
                   min={"cpu": 50_000, "memory": 100 << 30})
    p.on_quota_add("team-a-2", parent="team-a", max={"cpu": 120_000, "memory": 300 << 30},
                   min={"cpu": 50_000, "memory": 100 << 30}, allow_lent=False)
    p.on_quota_add("team-b", max={"cpu": 90_000, "memory": 200 << 30}, min={"cpu": 60_000, "memory": 100 << 30})
    return p


def pod_quotas(c, p):
    names = [None, "team-a-1", "team-a-2", "team-b"]
    out = []
    for i in range(len(c.pods)):
        q = names[(i * 7 + i // 5) % 4]
        req = {"cpu": int(c.pods["requests"][i, 0]), "memory": int(c.pods["requests"][i, 1])}
        out.append((q, req, i % 3 == 0))
        if q:
            p.on_pod_add(q, req, assigned=False)   # pending pods count in request (OnPodAdd)
    p.refresh_runtime()
    return out


def sequential(engine, p, pods, pq, seq):
    """The reference's order, one pod at a time: PreFilter, node loop, Reserve."""
    nodes, codes = np.full(len(pods), -1), []
    for i in range(len(pods)):
        q, req, np_ = pq[i]
        st = p.pre_filter(q, req, np_)
        codes.append((st.code, st.message))
        if st.is_success():
            r = engine.schedule(pods[i:i + 1], seq[i:i + 1])
            nodes[i] = r["node"][0]
            if nodes[i] >= 0:
                p.reserve_pod(q, req, np_)
    return nodes, codes


def oracle_tree():
    """The same forest in the Python restatement (oracle/quota.py)."""
    from oracle import quota as oq
    t = oq.QuotaTree({"cpu": 400_000, "memory": 800 << 30})
    t.add(oq.Quota("team-a", max={"cpu": 250_000, "memory": 600 << 30}, min={"cpu": 100_000, "memory": 200 << 30}))
    t.add(oq.Quota("team-a-1", parent="team-a", max={"cpu": 150_000, "memory": 400 << 30},
                   min={"cpu": 50_000, "memory": 100 << 30}))
    t.add(oq.Quota("team-a-2", parent="team-a", max={"cpu": 120_000, "memory": 300 << 30},
                   min={"cpu": 50_000, "memory": 100 << 30}, allow_lent=False))
    t.add(oq.Quota("team-b", max={"cpu": 90_000, "memory": 200 << 30}, min={"cpu": 60_000, "memory": 100 << 30}))
    return t


def sequential_oracle(engine, pods, pq, seq, check_parent=True):
    """One pod at a time with the quota gate of oracle/quota.py (independent of libgpuscore's gs_quota_*)."""
    from oracle import quota as oq
    t = oracle_tree()
    for q, req, _ in pq:
        if q:
            t.add_pod(q, req, assigned=False)
    t.refresh()
    nodes, codes = np.full(len(pods), -1), []
    for i in range(len(pods)):
        q, req, np_ = pq[i]
        code = oq.pre_filter(t, q, req, non_preemptible=np_, check_parent=check_parent)[0]
        codes.append("Success" if code == "Success" else "Unschedulable")
        if code == "Success":
            nodes[i] = engine.schedule(pods[i:i + 1], seq[i:i + 1])["node"][0]
            if nodes[i] >= 0 and q:
                name = q
                while name != oq.ROOT:
                    a = t.quotas[name]
                    a.used = {k: a.used.get(k, 0) + req.get(k, 0) for k in set(a.used) | set(req)}
                    if np_:
                        a.non_preemptible_used = {k: a.non_preemptible_used.get(k, 0) + req.get(k, 0)
                                                  for k in set(a.non_preemptible_used) | set(req)}
                    name = a.parent
    return nodes, codes
