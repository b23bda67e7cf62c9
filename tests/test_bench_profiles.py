"""bench.py's roofline `traffic` comes from the committed PMC profiles: the default files must exist, name
the bench's own default workloads, and hold the dominant kernel of each line (CPU only: JSON lookups)."""
import bench


def test_default_traffic_profiles_resolve():
    kw = bench.pmc_traffic(bench.TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=1_000_000, seed=20250905)
    dd = bench.pmc_traffic(bench.TRAFFIC_DEDUP, 'dd_transform_kernel', rows_per_gpu=500_000_000, seed=20250905)
    assert kw and kw > 2_000_000_000
    assert dd and dd > 40_000_000_000


def test_traffic_lookup_refuses_other_workloads():
    assert bench.pmc_traffic(bench.TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=10_000, seed=20250905) is None
    assert bench.pmc_traffic(bench.TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=1_000_000, seed=1) is None
    assert bench.pmc_traffic('none', 'kw_filter_kernel') is None
