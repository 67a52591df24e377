"""CPU tests of bench.py's measurement bookkeeping: roofline.traffic comes from the committed
rocprofv3 PMC summary only when it was collected on this very library build, for this kernel and
block count (never a stale figure), and the committed summary covers the kernels the default bench
line names."""
import json

import bench


def test_load_traffic_matches_build_kernel_and_blocks(tmp_path):
    sha = bench.lib_sha256()
    path = tmp_path / "pmc.json"
    path.write_text(json.dumps({"tag": "t", "lib_sha256": sha, "kernels": {
        "rs_wg_encode_kernel<6>": {"blocks": 1 << 20, "hbm_bytes_per_launch": 532219648.0}}}))
    v, src = bench.load_traffic("rs_wg_encode_kernel<6>", 1 << 20, path=str(path))
    assert v == 532219648 and "same library build" in src
    assert bench.load_traffic("rs_wg_encode_kernel<6>", 1 << 19, path=str(path))[0] is None  # other size
    assert bench.load_traffic("rs_bs_encode_kernel<32>", 1 << 20, path=str(path))[0] is None  # other kernel
    path.write_text(json.dumps({"tag": "t", "lib_sha256": "0" * 64, "kernels": {
        "rs_wg_encode_kernel<6>": {"blocks": 1 << 20, "hbm_bytes_per_launch": 1.0}}}))
    v, src = bench.load_traffic("rs_wg_encode_kernel<6>", 1 << 20, path=str(path))
    assert v is None and "another build" in src
    assert bench.load_traffic("x", 1, path=str(tmp_path / "missing.json"))[0] is None


def test_committed_pmc_summary_covers_the_bench_kernels():
    pmc = json.load(open(bench.os.path.join(bench.ROOT, "profiles", "pmc_latest.json")))
    ks = pmc["kernels"]
    for name in ("rs_wg_encode_tk_kernel<6>", "rs_wg_decode_tk_kernel<6>"):  # the default bench line's kernels
        assert name in ks and ks[name]["blocks"] == 1 << 20
        assert ks[name]["hbm_bytes_per_launch"] > 0
    for v in ks.values():  # any other profiled workload (cfg5) on the same build: well-formed
        assert v["blocks"] > 0 and v["hbm_bytes_per_launch"] > 0
