"""bench.py's N > 1 line carries every key that makes the driver's 8-GPU run
decisive: the direct self-check, the untuned and tuned
schedule of cfg3, the bidirectional-ring and measured-link fractions, the
per-link rates of the xGMI probe and the host-inclusive 1 GiB rate.  The line
is composed by bench.compose_multi from the run's measurements; here it is
fed a mocked 8-GPU run (CPU only: the HBM byte model is the library's
RdcPlanHbmBytes, which needs no GPU)."""
import copy
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def mocked_ctx(gpus_here):
    S = 1 << 30
    return {"world": 8, "S": S, "count": S // 4, "esz": 4, "dtype": "float32", "dt_enum": 6, "buckets": 1,
            "unfused": False, "algo": "auto", "steps": 20, "wall": 20 * 3.0e-3, "kern_ms": 2.98,
            "timed_algo": "direct", "gpus_here": gpus_here,
            "probe": {"one_link_one_direction_GBps": 60.1, "all_links_egress_GBps": 380.5,
                      "pull_one_link_GBps": 58.0, "pull_all_links_GBps": 350.2, "bytes_per_target": 256 << 20},
            "tuned": {"chosen": {"schedule": "direct", "grid": 512}, "candidates": []},
            "direct_selfcheck": "passed", "untuned": {"schedule": "direct", "ms_per_step": 3.05},
            "host_1g": {"algbw_GBps_pcie_inclusive": 21.4, "ms_per_step": 50.2}}


def line_for(bench, ctx):
    from rdc_amd._lib import _LIB
    roof, algo, keys = bench.compose_multi(_LIB, ctx)
    line = {"roofline": roof, "value": 1.0}
    line.update(keys)
    return line, algo


def test_mocked_eight_gpu_line_has_every_decisive_key():
    bench = load_bench()
    line, algo = line_for(bench, mocked_ctx(gpus_here=8))
    assert algo == "direct"
    assert bench.missing_multi_keys(line, need_values=True) == [], line
    r = line["roofline"]
    # busbw = S / t x 2(n-1)/n over the kernel time; against 153.6 GB/s and the probe's all-links rate
    busbw = (1 << 30) / 2.98e-3 / 1e9 * 14 / 8
    assert abs(r["frac_of_bidir_ring_roofline"] - round(busbw / 153.6, 4)) < 1e-4
    assert abs(r["frac_of_measured"] - round(busbw / 380.5, 4)) < 1e-4
    assert r["hbm"]["read_bytes_per_rank"] == 1 << 30 and r["hbm"]["write_bytes_per_rank"] == 1 << 30
    assert line["cfg3_schedule"]["untuned"]["schedule"] == "direct"
    assert line["cfg3_schedule"]["tuned"]["source"] == "RdcCommAutotune on this node"
    assert line["xgmi_link_rates"]["all_links_egress_GBps"] == 380.5


def test_shared_gpu_line_keeps_the_keys_with_null_link_fractions():
    bench = load_bench()
    line, _ = line_for(bench, mocked_ctx(gpus_here=1))
    assert bench.missing_multi_keys(line) == [], line   # present ...
    nulls = bench.missing_multi_keys(line, need_values=True)
    assert nulls == ["roofline.frac_of_bidir_ring_roofline", "roofline.frac_of_measured"], nulls  # ... null
    assert line["roofline"]["bound"] == "shared-hbm"


def test_a_missing_key_is_reported():
    bench = load_bench()
    line, _ = line_for(bench, mocked_ctx(gpus_here=8))
    for path in bench.REQUIRED_MULTI_KEYS:
        broken = copy.deepcopy(line)
        cur = broken
        parts = path.split(".")
        for p in parts[:-1]:
            cur = cur[p]
        del cur[parts[-1]]
        assert bench.missing_multi_keys(broken) == [path], path
    # no probe, no untuned timing, no host leg: keys stay, values null
    ctx = mocked_ctx(gpus_here=8)
    ctx.update({"probe": {"error": "timed out"}, "untuned": None, "host_1g": None})
    line, _ = line_for(bench, ctx)
    assert bench.missing_multi_keys(line) == []
    assert set(bench.missing_multi_keys(line, need_values=True)) == {
        "cfg3_schedule.untuned.schedule", "cfg3_schedule.untuned.ms_per_step", "roofline.frac_of_measured",
        "xgmi_link_rates.one_link_one_direction_GBps", "xgmi_link_rates.all_links_egress_GBps",
        "host_inclusive_1GiB.algbw_GBps_pcie_inclusive"}


def test_main_composes_the_line_with_compose_multi():
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "roof, algo_name, multi_keys = compose_multi(_LIB, ctx)" in src
    assert "out.update(multi_keys)" in src
    assert '"host_1g": extra.get("host_1GiB")' in src
