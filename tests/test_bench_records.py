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


def test_pmc_merge_keeps_each_kernels_in_step_entry():
    """tools/pmc_summary.py merge_latest: profiles of one build merge, each kernel keeping the run
    whose bench step launched it; another build replaces the file."""
    from tools.pmc_summary import merge_latest

    head = {"rs_wg_decode_tk_kernel<6>": {"blocks": 1 << 20, "hbm_bytes_per_launch": 567e6, "in_step_launches": 9466},
            "rs_bs_decode_kernel<32>": {"blocks": 1 << 20, "hbm_bytes_per_launch": 510e6}}
    cfg5 = {"rs_wg_decode_tk_kernel<6>": {"blocks": 1 << 20, "hbm_bytes_per_launch": 534e6},
            "rs_bs_decode_kernel<32>": {"blocks": 1 << 20, "hbm_bytes_per_launch": 543e6, "in_step_launches": 7690}}
    a = merge_latest({}, head, "s" * 64, "r6fin")
    b = merge_latest(a, cfg5, "s" * 64, "r6fin_cfg5")
    assert b["tag"] == "r6fin+r6fin_cfg5"
    assert b["kernels"]["rs_wg_decode_tk_kernel<6>"]["hbm_bytes_per_launch"] == 567e6  # the headline run's
    assert b["kernels"]["rs_bs_decode_kernel<32>"]["hbm_bytes_per_launch"] == 543e6  # the cfg5 run's
    c = merge_latest(b, cfg5, "t" * 64, "r7")
    assert c["tag"] == "r7" and c["kernels"] == cfg5


def test_committed_pmc_headline_entries_are_in_step():
    """The committed summary's headline kernels come from the headline profile: in-step launches, and
    the 1-error decode's traffic carries its 2^20 one-byte write-backs (above the algorithmic bytes)."""
    ks = json.load(open(bench.os.path.join(bench.ROOT, "profiles", "pmc_latest.json")))["kernels"]
    for name in ("rs_wg_encode_tk_kernel<6>", "rs_wg_decode_tk_kernel<6>"):
        assert ks[name].get("in_step_launches", 0) > 0
    assert ks["rs_wg_decode_tk_kernel<6>"]["hbm_bytes_per_launch"] > 1.05 * 528482304


def test_config_lines_carry_cold_per_leg_fractions():
    """tools/bench_configs.py's lines (bench.py `configs`): one fraction per leg, the cold-set count,
    no max-over-legs figure (round 6: roofline_frac_best dropped); cfg5_step's in-step fields."""
    from tools.bench_configs import config_line, rotation_sets, step_line

    nb = 1 << 20
    assert rotation_sets(nb * 504) == 3 and rotation_sets(nb * 478) == 3  # RS(255,249), RS(255,223)
    assert rotation_sets(nb * 8187) == 1  # cfg4: one set is already 32x the Infinity Cache
    line = config_line("cfg5 rs255_t16 bs4096", nb, 255, 223, "rs255-bs-byte-lds", 3, 0.104, 0.100, 0.112, True)
    assert "roofline_frac_best" not in line and line["cold_sets"] == 3
    assert abs(line["roofline_frac_encode"] - 478 * nb / 0.104e-3 / 8e12) < 1e-4
    assert abs(line["roofline_frac_decode_1err"] - 478 * nb / 0.112e-3 / 8e12) < 1e-4
    crc = config_line("cfg4 crc", nb, 4096, 4092, "crc", 1, 1.5, 1.5)
    assert "decode_1err_ms" not in crc and "roofline_frac_decode_1err" not in crc
    st = step_line(4096, 16, nb, 255, 223, 20, 0.104, 0.112, 0.03, 0.25, True)
    assert st["in_step_frac"]["encode"] == round(478 * nb / 0.104e-3 / 8e12, 4)
    assert st["in_step_frac"]["decode"] == round(478 * nb / 0.112e-3 / 8e12, 4)
    assert st["kernels_ms"] == {"encode": 0.104, "inject": 0.03, "decode": 0.112} and st["verified"]
    assert abs(st["GiBps"] - 2 * 478 * nb / 0.25e-3 / 2**30) < 1e-2


def test_cfg1_leg_parses_the_harness_lines(monkeypatch, tmp_path):
    """bench.py's cfg1 object from tests/cpp/bench_blockdevice's JSON lines (the binary is stood in)."""
    import subprocess

    lines = [
        {"bench": "BM_BlockDevice_Read/rs_test/1", "iterations": 10, "us_per_call": 8.5, "BytesRead_per_s": 117647, "ok": True},
        {"bench": "BM_BlockDevice_Write/crc_test/256", "iterations": 10, "us_per_call": 30.0, "BytesWritten_per_s": 8533333,
         "ok": True},
        {"bench": "cfg1 rs255_t3 4096 blocks", "per_block_write_blocks_per_s": 60000, "per_block_read_blocks_per_s": 130000,
         "batched_write_blocks_per_s": 4.0e6, "batched_read_blocks_per_s": 5.0e6, "ok": True},
    ]

    class R:
        returncode = 0
        stdout = "\n".join(json.dumps(x) for x in lines) + "\n"
        stderr = ""

    monkeypatch.setattr(bench.os.path, "exists", lambda p: True)
    monkeypatch.setattr(subprocess, "run", lambda *a, **k: R())
    out = bench.cfg1_leg()
    assert out["sweep"]["rs"]["read_1"] == {"us_per_call": 8.5, "KiB_per_s": round(117647 / 1024, 1), "ok": True}
    assert out["sweep"]["crc"]["write_256"]["us_per_call"] == 30.0
    assert out["rs255_249_4096_blocks"]["per_block_read_blocks_per_s"] == 130000
    assert out["per_block_read_vs_reference_cpu"] == round(130000 / 95162, 2)
    assert out["reference_cpu"]["writeBlock_blocks_per_s"] == 2422
