"""GPU parity at the scan's capacity boundaries, forced small through the library's test overrides.

Each scratch region of a scan (csrc/kwmatch.hip launch_scan) has a capacity sized from the corpus; when a
region overflows, the scan either grows it and rescans, or defers the affected documents to the generic kernel.
The golden and the adversarial corpora rarely reach these paths, so here each capacity is set tiny
(KW_TEST_* overrides, honoured under KW_TEST_HOOKS=1, tests/conftest.py) on a fresh handle, and the results
must still equal the CPU oracle (match_keywords.py:155-180 per field) while the statistics show that the path
ran:

* KW_TEST_CAND_CAP   the filter's candidate regions overflow -> ST_CAND_OVERFLOW -> larger regions, rescan
* KW_TEST_ITEM_CAP   the probe's item regions overflow: the batches that do not fit defer their documents
                     (nothing reads items that were not written), then larger regions, rescan
* KW_TEST_ITEM_LIMIT the item index limit (2^32 in production) reached: no growth, the overflowing batches'
                     documents go to the generic kernel in the same scan
* KW_TEST_TASK_CAP   the verify / short / regex task queues overflow -> ST_TASK_OVERFLOW -> rescan
* KW_TEST_DSET_SIZE  the decided (doc, field, name) set fills -> ST_DSET_FULL -> rescan

and the scheduling knobs (KW_DEV=1) leave the results unchanged: the epilogue's regex tasks beside the verify /
short kernels or after them (KW_RX_SPLIT), at 1 or 4 waves a region, the side streams' priorities.
"""
import pytest

from advanced_scrapper_amd import _native

from tests.test_gpu_parity import _adversarial_strings, _compare, _golden_rows, _gpu_maps, _many_item_docs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def corpus(golden):
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    processed = golden.kb_processed()
    ckb = compile_kb(processed)
    texts, titles, _ = _golden_rows(golden)
    a_t, a_i = _adversarial_strings(ckb)
    m_t, m_i = _many_item_docs(ckb)
    names, kinds = synth.injectable_names(ckb)
    c = synth.generate(600, names, kinds, seed=31, doc_base=7000)
    return {'processed': processed, 'ckb': ckb,
            'texts': texts + a_t + m_t + c.texts(), 'titles': titles + a_i + m_i + c.titles()}


# Every capacity large (a scan of this corpus grows none of them): the reference point of each test below,
# which makes one capacity small and keeps the others large, so the statistics show that capacity's path alone
LARGE = {'KW_TEST_CAND_CAP': 1 << 20, 'KW_TEST_ITEM_CAP': 1 << 20, 'KW_TEST_TASK_CAP': 1 << 16,
         'KW_TEST_DSET_SIZE': 1 << 22}
CAUSES = _native.KW_RESCAN_REGIONS | _native.KW_RESCAN_TASK_QUEUES | _native.KW_RESCAN_DECIDED_SET


def _run(corpus, monkeypatch, large=True, **env):
    from advanced_scrapper_amd.matcher import GpuMatcher
    for k, v in {**(LARGE if large else {}), **env}.items():
        monkeypatch.setenv(k, str(v))
    m = GpuMatcher(corpus['ckb'])            # a fresh handle: its regions start at the forced sizes
    got = _gpu_maps(m, corpus['texts'], corpus['titles'])
    bad = _compare(corpus['processed'], corpus['texts'], corpus['titles'], got)
    st = m.stats()
    assert not bad, f"{env}: GPU differs from the oracle on docs {bad[:20]} (stats {st})"
    return st


@pytest.fixture(scope='module')
def natural(corpus):
    """The corpus with the library's own sizing (no overrides): its many-item documents grow buffers."""
    mp = pytest.MonkeyPatch()
    try:
        return _run(corpus, mp, large=False)
    finally:
        mp.undo()


@pytest.fixture(scope='module')
def baseline(corpus):
    """Every capacity large: no region, task queue or decided set overflows."""
    mp = pytest.MonkeyPatch()
    try:
        return _run(corpus, mp)
    finally:
        mp.undo()


def test_baseline_no_overrides(baseline, natural):
    assert natural['deferred_docs'] > 0 and natural['big_docs'] > 0
    # with every capacity large nothing overflows: each test below must add its own cause
    assert not baseline['rescan_causes'] & CAUSES, baseline


def test_candidate_region_overflow_rescans(corpus, baseline, monkeypatch):
    st = _run(corpus, monkeypatch, KW_TEST_CAND_CAP=16)
    assert st['rescan_causes'] & _native.KW_RESCAN_REGIONS


def test_item_region_overflow_defers_then_grows(corpus, baseline, monkeypatch):
    st = _run(corpus, monkeypatch, KW_TEST_ITEM_CAP=8)
    assert st['rescan_causes'] & _native.KW_RESCAN_REGIONS


def test_item_index_limit_defers_to_generic(corpus, baseline, monkeypatch):
    """No growth past the item index limit: the documents of every batch that did not fit its region are
    finished by the generic kernel in the same scan (results exact, deferred_docs > 0)."""
    st = _run(corpus, monkeypatch, KW_TEST_ITEM_LIMIT=1024)
    assert st['deferred_docs'] > baseline['deferred_docs']


def test_task_queue_overflow_rescans(corpus, baseline, monkeypatch):
    st = _run(corpus, monkeypatch, KW_TEST_TASK_CAP=2)
    assert st['rescan_causes'] & _native.KW_RESCAN_TASK_QUEUES


def test_decided_set_full_rescans(corpus, baseline, monkeypatch):
    st = _run(corpus, monkeypatch, KW_TEST_DSET_SIZE=4)
    assert st['rescan_causes'] & _native.KW_RESCAN_DECIDED_SET


def test_overrides_ignored_without_the_gate(corpus, natural, monkeypatch):
    """A production process (no KW_TEST_HOOKS) ignores the overrides: the library's own sizing's statistics."""
    monkeypatch.delenv('KW_TEST_HOOKS', raising=False)
    st = _run(corpus, monkeypatch, large=False, KW_TEST_CAND_CAP=16, KW_TEST_TASK_CAP=2)
    assert st == natural


@pytest.mark.parametrize('env', [{'KW_RX_SPLIT': 0}, {'KW_RX_SPLIT': 1, 'KW_RX_EARLY_G': 1, 'KW_SIDE_PRIO': 0},
                                 {'KW_RX_SPLIT': 1, 'KW_RX_EARLY_G': 4, 'KW_SIDE_PRIO': 3}])
def test_regex_task_split_and_stream_priorities(corpus, natural, monkeypatch, env):
    """The regex tasks the epilogue queued run beside the verify / short kernels (phase 1, up to the count each
    epilogue wave wrote) or after them with the rest (phase 2 / 0): every task exactly once either way."""
    monkeypatch.setenv('KW_DEV', '1')
    st = _run(corpus, monkeypatch, large=False, **env)
    assert st['regex_searches'] == natural['regex_searches'] and st['deferred_docs'] == natural['deferred_docs']
