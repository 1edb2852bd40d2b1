"""bench.py's reporting helpers on the CPU: the roofline's `traffic` comes
from the committed PMC summary (profiles/pmc_summary.json), and the CPU
baseline runs on every host core the process may use."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_committed_pmc_summary_gives_traffic_for_the_encode_kernels():
    summary = json.load(open(os.path.join(ROOT, "profiles", "pmc_summary.json")))
    assert "bytes_per_unit" in summary, "commit the file scripts/pmc_summary.py writes, not its stdout"
    for kernel, units in (("huff", 56_700_000), ("fdct", 333 * 3840 * 2160)):
        t = bench.pmc_traffic(kernel, units)
        assert t is not None and t > 0, kernel
    # k_huff: measured HBM bytes within 1.0x-1.5x of its ~74 algorithmic B per block-trial
    assert 74 <= summary["bytes_per_unit"]["huff"] <= 111
    # k_fdct_color: 3 B/px pixel reads + candidate lists
    assert 3.0 <= summary["bytes_per_unit"]["fdct"] <= 6.0


def test_pmc_bytes_per_unit_reads_both_summary_forms():
    file_form = {"bytes_per_unit": {"huff": 82.5}}
    kernel_form = {"icx::k_huff": {"hbm_bytes_per_unit": 82.5}, "icx::k_fdct_color<true>": {"hbm_bytes_per_unit": 4.27},
                   "icx::k_other": {"hbm_bytes_per_unit": 1.0}}
    assert bench.pmc_bytes_per_unit(file_form) == {"huff": 82.5}
    assert bench.pmc_bytes_per_unit(kernel_form) == {"huff": 82.5, "fdct": 4.27}


def test_host_cores_is_the_usable_core_count():
    n, how = bench.host_cores()
    assert 1 <= n <= len(os.sched_getaffinity(0))
    assert how in ("sched_getaffinity", "cgroup cpu.max quota")
