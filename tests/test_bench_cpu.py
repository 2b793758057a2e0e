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
                          (bench.gru_bwd_kernel(True)[2], ()), ("gru_fwd_x6", ())):
        traffic, src = bench.pmc_traffic_per_launch(prefix, extra)
        assert src == os.path.join("profiles", bench.PMC_SUMMARY)
        assert traffic is not None and traffic > 1e8, prefix
