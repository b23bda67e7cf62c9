"""Pin the oracle: partial_ratio restatement self-consistency + golden vectors."""
import random

import numpy as np
import pandas as pd
import pytest
from dateutil import parser

from oracle import kwmatch_oracle as orc


def test_float_rule_equals_integer_rule():
    # score > 95 with score = 100*(1 - d/L) (or 100 - 100*d/L) <=> 20*d < L
    for L in range(1, 300):
        for d in range(0, L + 1):
            s1 = 100.0 * (1.0 - d / L)
            s2 = 100.0 - 100.0 * d / L
            want = 20 * d < L
            assert (s1 > 95) == want, (d, L)
            assert (s2 > 95) == want, (d, L)


@pytest.mark.parametrize('seed', [1, 2])
def test_partial_ratio_brute_fast_decide_agree(seed):
    rng = random.Random(seed)
    alpha = 'abcdé ,.'
    for _ in range(3000):
        a = ''.join(rng.choice(alpha) for _ in range(rng.randint(0, 40)))
        b = ''.join(rng.choice(alpha) for _ in range(rng.randint(0, 40)))
        if rng.random() < 0.6 and len(b) > 2:
            i = rng.randint(0, len(b) - 1)
            j = rng.randint(i, len(b))
            piece = list(b[i:j])
            for _k in range(rng.randint(0, 3)):   # a few indels
                if piece and rng.random() < 0.5:
                    del piece[rng.randrange(len(piece))]
                else:
                    piece.insert(rng.randint(0, len(piece)), rng.choice(alpha))
            a = a[:rng.randint(0, len(a))] + ''.join(piece) + a[rng.randint(0, len(a)):]
        s_b = orc.partial_ratio_score(a, b, brute=True)
        s_f = orc.partial_ratio_score(a, b)
        assert s_b == s_f, (a, b)
        assert (s_b > 95) == orc.partial_ratio_gt95(a, b), (a, b, s_b)
        assert orc.partial_ratio_score(a, b) == orc.partial_ratio_score(b, a)


@pytest.mark.parametrize('seed', [3, 4])
def test_long_needles_decide_many_equals_brute(seed):
    """Names of 21..64 code points (the pigeonhole-covered full windows) inside longer texts with up to 6
    indels, through pr_decide_many (the per-text occurrence index) and pr_decide, against the brute-force
    window-family score."""
    rng = random.Random(seed)
    alpha = 'abcdeé ,.AB'
    for _ in range(60):
        names = []
        for _k in range(8):
            names.append(''.join(rng.choice(alpha) for _ in range(rng.randint(21, 64))))
        text = ''.join(rng.choice(alpha) for _ in range(rng.randint(60, 260)))
        for nm in rng.sample(names, 3):
            piece = list(nm)
            for _k in range(rng.randint(0, 6)):
                if rng.random() < 0.5:
                    del piece[rng.randrange(len(piece))]
                else:
                    piece.insert(rng.randint(0, len(piece)), rng.choice(alpha))
            cut = rng.randint(0, len(text))
            if rng.random() < 0.2:
                cut = rng.choice((0, len(text)))
                piece = piece[rng.randint(0, 5):] if cut == 0 else piece[:len(piece) - rng.randint(0, 5)]
            text = text[:cut] + ''.join(piece) + text[cut:]
        if rng.random() < 0.2:
            text = text[:rng.randint(20, 64)]        # texts shorter than some names swap roles
        many = orc.NameSet(names).decide(text)
        for nm, got in zip(names, many):
            want = orc.partial_ratio_score(text, nm, brute=True) > 95
            assert bool(got) == want, (text, nm)
            assert orc.partial_ratio_gt95(text, nm) == want, (text, nm)


def test_partial_ratio_known_properties():
    assert orc.partial_ratio_score('', '') == 100.0
    assert orc.partial_ratio_score('abc', '') == 0.0
    assert orc.partial_ratio_score('xx Apple Inc yy', 'Apple Inc') == 100.0
    # m <= 10: only an exact substring passes
    assert not orc.partial_ratio_gt95('xx Apple Ink yy', 'Apple Inc')
    # 11..20: one deletion at the text edge passes (d = 1 edge window)
    assert orc.partial_ratio_gt95('pple Computer Inc. rest of text', 'Apple Computer Inc.')
    assert not orc.partial_ratio_gt95('rest pple Computer Inc. rest', 'Apple Computer Inc.')
    # >= 21: one interior indel pair passes
    assert orc.partial_ratio_gt95('aa Walt Disney Parks and Resort U.S. bb', 'Walt Disney Parks and Resorts U.S.')
    # text shorter than the name swaps roles
    assert orc.partial_ratio_gt95('nan', 'Capital One Financial')
    assert orc.partial_ratio_gt95('Walt Disney Company', 'The Walt Disney Company')


def _rows(frame):
    out = []
    for _i, row in frame.iterrows():
        text = str(row['article_text']) if row['article_text'] else ""
        title = str(row['title']) if row['title'] else ""
        date = parser.parse(str(row['date_time'])) if pd.notna(row['date_time']) else None
        out.append((text, title, date))
    return out


def test_oracle_reproduces_reference_golden(golden):
    """oracle.ticker_matches == what the reference's process_chunk built (all golden rows)."""
    frame = golden.articles_frame()
    want = golden.matches()
    oracle = orc.Oracle(golden.kb_processed())
    rows = _rows(frame)
    assert len(rows) == len(want)
    bad = []
    for i, (text, title, date) in enumerate(rows):
        got = oracle.ticker_matches(text, title, date)
        if got != want[i] or list(got) != list(want[i]):
            bad.append(i)
        else:   # dict order inside each ticker too
            for t in got:
                assert list(got[t]['text']) == list(want[i][t]['text'])
                assert list(got[t]['title']) == list(want[i][t]['title'])
    assert not bad, f"oracle differs from the reference on rows {bad[:10]}"
