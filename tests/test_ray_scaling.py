"""Ray scaling policy (runtime/ray_scaling.py; reference runtime/ray/scaling_policy.py) against
canned Ray dashboard responses: pending task / placement-group shapes become resource
demands (bounded), raylet reports become node states, dead raylets lost nodes."""
from cloudtik_amd.core import runtime_factory as rf
from cloudtik_amd.runtime.ray_scaling import MAX_DEMAND, RayScalingPolicy, resource_demands

STATUS = {"data": {"clusterStatus": {"loadMetricsReport": {
    "resourceDemand": [[{"CPU": 1.0, "GPU": 1.0}, 3], [{"CPU": 8.0}, 2]],
    "pgDemand": [[[{"GPU": 8.0}, {"GPU": 8.0}], 1]]}}}}
NODES = {"data": {"summary": [
    {"raylet": {"nodeManagerAddress": "10.0.0.1", "state": "ALIVE", "resourcesTotal": {"CPU": 128, "GPU": 8,
                                                                                       "node:10.0.0.1": 1},
                "resourcesAvailable": {"CPU": 100, "GPU": 2}}},
    {"raylet": {"nodeManagerAddress": "10.0.0.2", "state": "DEAD", "resourcesTotal": {"CPU": 128}}}]}}


def _fetch(path):
    return STATUS if path.startswith("api/cluster_status") else NODES


def test_demands_nodes_and_lost():
    cfg = {"runtime": {"ray": {"auto_scaling": True}}}
    st = RayScalingPolicy(cfg, "10.0.0.1", _fetch).get_scaling_state()
    d = st.autoscaling_instructions["resource_demands"]
    assert d.count({"CPU": 1.0, "GPU": 1.0}) == 3 and d.count({"CPU": 8.0}) == 2 and d.count({"GPU": 8.0}) == 2
    n = st.node_resource_states["10.0.0.1"]
    assert n["total"] == {"CPU": 128.0, "GPU": 8.0} and n["used"]["GPU"] == 6.0
    assert st.lost_nodes == {"10.0.0.2": "10.0.0.2"}
    off = RayScalingPolicy({"runtime": {"ray": {}}}, "h", _fetch).get_scaling_state()
    assert off.autoscaling_instructions is None


def test_demands_are_bounded_and_runtime_hook():
    big = {"resourceDemand": [[{"CPU": 1}, 5000]]}
    assert len(resource_demands(big)) == MAX_DEMAND
    rt = rf.get_runtime("ray", {"auto_scaling": True})
    assert isinstance(rt.get_scaling_policy({"runtime": {"ray": {"auto_scaling": True}}}, "h"), RayScalingPolicy)
    assert rf.get_runtime("ray", {}).get_scaling_policy({"runtime": {"ray": {}}}, "h") is None
