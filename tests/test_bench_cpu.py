"""bench.py host-side pieces that need no GPU: the committed PMC summary it prices HBM
traffic from exists and has the kernels the JSON line reports."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_pmc_summary_is_committed_and_covers_the_reported_kernels():
    import bench
    assert os.path.exists(os.path.join(REPO, "profiles", bench.PMC_SUMMARY))
    # the kernels of the default configuration (bench.gru_bwd_kernel / gru_fwd_kernel name them)
    for prefix, extra in (("gemm", ("splitk_reduce_kernel",)),
                          (bench.gru_bwd_kernel(True)[2], ()), (bench.gru_fwd_kernel(True)[2], ())):
        traffic, src = bench.pmc_traffic_per_launch(prefix, extra)
        assert src == os.path.join("profiles", bench.PMC_SUMMARY)
        assert traffic is not None and traffic > 1e8, prefix


def test_bench_probes_every_recurrence_entry_point():
    """bench.py times the GRU recurrences by wrapping the C-ABI entry points ops.py calls: every
    ds2_gru_fwd* / ds2_gru_bwd* name the GRU layer calls must be one the probes wrap (a renamed
    entry point silently dropped the backward from the bench line once)."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "deepspeech.pytorch_amd", "ds2amd", "ops.py")).read()
    called = set(re.findall(r'"(ds2_gru_(?:fwd|bwd)\w*)"', src)) - {
        "ds2_gru_fwd_workspace_size", "ds2_gru_bwd_workspace_size", "ds2_gru_bwd_grid"}
    bench_src = open(os.path.join(root, "bench.py")).read()
    probed = set(re.findall(r'"(ds2_gru_(?:fwd|bwd)\w*)"', bench_src))
    assert called and called <= probed, sorted(called - probed)
