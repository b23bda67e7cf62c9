"""bench.py's roofline `traffic` comes from the committed PMC profiles: the default files must exist, name
the bench's own default workloads and the library they profiled, and hold the dominant kernel of each line
(CPU only: JSON lookups)."""
import json

import bench


def _sha(path):
    return json.load(open(path))['workload']['library_sha256']


def test_default_traffic_profiles_resolve():
    kw_sha, dd_sha = _sha(bench.TRAFFIC_KW), _sha(bench.TRAFFIC_DEDUP)
    kw = bench.pmc_traffic(bench.TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=1_000_000, seed=20250905,
                           library_sha256=kw_sha)
    dd = bench.pmc_traffic(bench.TRAFFIC_DEDUP, 'dd_transform_kernel', rows_per_gpu=500_000_000, seed=20250905,
                           library_sha256=dd_sha)
    assert kw and kw > 2_000_000_000
    assert dd and dd > 40_000_000_000
    step = bench.pmc_step_traffic(bench.TRAFFIC_KW, docs_per_gpu=1_000_000, seed=20250905, library_sha256=kw_sha)
    assert step and step > kw
    # every kernel of the library counts, template instances included ("void kw::kw_epi_flat_kernel<true>(...)")
    ks = json.load(open(bench.TRAFFIC_KW))['kernels']
    want = sum(v['hbm_bytes_per_launch'] * v.get('launches_per_step', 1) for k, v in ks.items() if 'kw::' in k)
    assert any(k.startswith('void kw::') for k in ks) and step == int(want)
    assert all(v.get('launches_per_step', 1) in (1.0, 2.0) for k, v in ks.items() if 'kw::' in k)
    c4 = bench.pmc_traffic(bench.TRAFFIC_C4, 'kw_filter_kernel', docs_per_gpu=1_000_000, seed=20250905,
                           workload='kb50k', library_sha256=_sha(bench.TRAFFIC_C4))
    assert c4 and c4 > 2_000_000_000


def test_traffic_lookup_refuses_other_workloads_and_libraries():
    sha = _sha(bench.TRAFFIC_KW)
    assert bench.pmc_traffic(bench.TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=10_000, seed=20250905,
                             library_sha256=sha) is None
    assert bench.pmc_traffic(bench.TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=1_000_000, seed=1,
                             library_sha256=sha) is None
    # a profile of another build prices nothing
    assert bench.pmc_traffic(bench.TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=1_000_000, seed=20250905,
                             library_sha256='0' * 64) is None
    assert bench.pmc_step_traffic(bench.TRAFFIC_KW, docs_per_gpu=1_000_000, seed=20250905,
                                  library_sha256='0' * 64) is None
    assert bench.pmc_traffic('none', 'kw_filter_kernel') is None


def test_shard_plan_config3_and_labels():
    import argparse
    a = argparse.Namespace(docs_per_gpu=None, total_docs=None)
    assert bench.shard_plan(a, 0, 1) == (0, 1_000_000, 1_000_000, 'strong')
    plans = [bench.shard_plan(a, r, 8) for r in range(8)]
    assert [p[0] for p in plans] == [r * 1_250_000 for r in range(8)]
    assert sum(p[1] for p in plans) == 10_000_000 and {p[2] for p in plans} == {10_000_000}
    plans = [bench.shard_plan(a, r, 3) for r in range(3)]     # ragged: the last shard takes the remainder
    assert sum(p[1] for p in plans) == 10_000_000 and plans[2][0] + plans[2][1] == 10_000_000
    assert bench.workload_label(10_000_000, 8) == 'config 3' and bench.workload_label(10_000_000, 1) == 'config 3'
    assert bench.workload_label(1_000_000, 1) == 'config 2' and bench.workload_label(8_000_000, 8) != 'config 3'
    w = argparse.Namespace(docs_per_gpu=1000, total_docs=None)
    assert bench.shard_plan(w, 3, 4) == (3000, 1000, 4000, 'weak')


def test_bench_kb_is_the_products_loader_on_the_reference_files(tmp_path, golden):
    assert bench.load_kb(str(tmp_path / 'ticker')) == golden.kb_processed()
