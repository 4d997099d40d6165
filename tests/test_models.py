from test_nccl_p2p_amd.models import PRESETS, ParallelConfig, traffic_for


def test_pp_activation_size():
    t = traffic_for(PRESETS["llama3-70b"], ParallelConfig(pp=8, micro_batch=1, seq_len=4096))
    f = t["flows"][0]
    assert f["pattern"] == "pp-activation" and f["bytes"] == 4096 * 8192 * 2 and f["mode"] == "ring"


def test_moe_dispatch_and_cp():
    t = traffic_for(PRESETS["mixtral-8x7b"], ParallelConfig(ep=8, cp=2, seq_len=8192))
    kinds = {f["pattern"] for f in t["flows"]}
    assert kinds == {"ep-dispatch", "cp-kv-ring"}
    assert all(s & (s - 1) == 0 for s in t["sweep"])
    assert any("--mode allpairs" in c for c in t["commands"])
