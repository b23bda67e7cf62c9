"""Seeded synthetic Wikidata-style ticker knowledge base (config 4).

The reference's KB is ``info/ticker/*.json`` turned into ``processed_data`` by
``read_and_process_json_files`` (match_keywords.py:68-120): ticker ->
attribute (``id_label, ticker, aliases, products, subsidiaries,
owned_entities, ceos, board_members``, :77-84) -> name -> (start, end)
period.  Config 4 asks for ~50k patterns "from the same generator (names +
products + people), all <= 64 code points".  This module produces exactly that
dict, shaped like the real 216-ticker KB (tests/golden): company names with
legal suffixes (``Inc.``, ``S.A.``, ``Co.,Ltd.`` -- regex ``.`` wildcards),
``Brand+`` products (a ``+`` quantifier), ``xyz.com`` domains, uppercase
aliases and tickers (the ``\\b`` branch), people with initials, ~1 % non-ASCII
names, single-letter tickers and lowercase products (the never-matching
classes) and ~25 % of names carrying Start/End periods.

Pure function of (n_tickers, seed); no file or network access.
"""
from __future__ import annotations

import random
from datetime import datetime, timedelta
from typing import Dict, Tuple

ATTRS = ('id_label', 'ticker', 'aliases', 'products', 'subsidiaries', 'owned_entities', 'ceos', 'board_members')

_SYL = ("ac ad al am an ar as at ba be bi bo ca ce ci co da de di do ea el em en er es et fa fe fi fo ga ge gi go "
        "ha he hi ho ia ic id il im in io is it ka ke ki ko la le li lo lu ma me mi mo mu na ne ni no nu ol om on "
        "or os pa pe pi po ra re ri ro ru sa se si so su ta te ti to tu va ve vi vo xa xe za ze zi zo qu tr st br "
        "cr gr pr pl cl fl gl bl sk sp vr dr").split()
_END = "n x l r s m t k d co ra ix on ex ia us io um ar is os ta".split()
_FIRST = ("James John Robert Michael William David Richard Joseph Thomas Charles Mary Patricia Jennifer Linda "
          "Elizabeth Barbara Susan Jessica Sarah Karen Nancy Lisa Betty Margaret Sandra Ashley Kimberly Emily "
          "Donna Michelle Daniel Matthew Anthony Mark Donald Steven Paul Andrew Joshua Kenneth Kevin Brian George "
          "Timothy Ronald Edward Jason Jeffrey Ryan Jacob Gary Nicholas Eric Jonathan Stephen Larry Justin Scott "
          "Brandon Benjamin Samuel Gregory Alexander Frank Patrick Raymond Jack Dennis Jerry Tyler Aaron Jose Adam "
          "Nathan Henry Douglas Zachary Peter Kyle Ethan Walter Noah Jeremy Christian Keith Roger Terry Gerald "
          "Harold Sean Austin Carl Arthur Lawrence Dylan Jesse Jordan Bryan Billy Joe Bruce Gabriel Logan Albert "
          "Willie Alan Juan Wayne Elijah Randy Roy Vincent Ralph Eugene Russell Bobby Mason Philip Louis Ursula "
          "Indra Satya Sundar Mukesh Ratan Akio Masayoshi Yuki Wei Ming Jing Priya Anil Rajiv Hans Klaus Pierre "
          "Amélie François Søren José Zoë").split()
_CO_SUFFIX = ("Inc. Corporation Corp. Holdings Group Ltd. LLC Co. plc AG S.A. Limited International Technologies "
              "Systems Partners Capital Energy Financial Industries Brands Labs Networks Solutions Therapeutics "
              "Pharmaceuticals Bancorp Resources Motors Media Entertainment Foods Realty Trust").split()
_REGION = ("Germany Japan UK Canada Brasil France China India Australia Europe Italy Spain Korea Mexico Ireland "
           "Singapore Netherlands Sweden Switzerland Asia Africa Nordic Iberia Benelux México Zürich Québec").split()
_P_SUFFIX = "Pro Max Cloud One Plus Go Studio Hub Pay Connect 360 Lite Edge AI Prime Home Air Link Care Works".split()
_UNIT = "Center Tower Park Plaza Arena Field Campus Labs Foundation Institute Ventures Studios Bank Fund".split()
_NONASCII = "é ü ö ñ ç ø å".split()


def _word(r: random.Random, lo: int = 2, hi: int = 3) -> str:
    w = ''.join(r.choice(_SYL) for _ in range(r.randint(lo, hi))) + r.choice(_END)
    if r.random() < 0.02:   # a non-ASCII letter somewhere inside
        i = r.randrange(1, len(w))
        w = w[:i] + r.choice(_NONASCII) + w[i + 1:]
    return w.capitalize()


def _person(r: random.Random) -> str:
    first, last = r.choice(_FIRST), _word(r, 1, 2)
    k = r.random()
    if k < 0.55:
        return f"{first} {last}"
    if k < 0.80:
        return f"{first} {chr(65 + r.randrange(26))}. {last}"
    if k < 0.90:
        return f"{chr(65 + r.randrange(26))}. {first} {last}"
    if k < 0.95:
        return f"{first} {last} Jr."
    return f"{first}-{r.choice(_FIRST)} {last}"


def _ticker_symbol(r: random.Random, used: set) -> str:
    while True:
        n = 1 if r.random() < 0.01 else r.choice((2, 3, 3, 4, 4, 4, 5))
        s = ''.join(chr(65 + r.randrange(26)) for _ in range(n))
        if s not in used:
            used.add(s)
            return s


def _period(r: random.Random) -> Tuple[object, object]:
    """(start, end) like extract_time_periods' output (match_keywords.py:40-65): ~75 % unbounded."""
    k = r.random()
    if k < 0.75:
        return (None, None)
    base = datetime(1980, 1, 1)
    a = base + timedelta(days=r.randrange(0, 16000))
    b = a + timedelta(days=r.randrange(30, 9000))
    if k < 0.85:
        return (a, None)
    if k < 0.92:
        return (None, b)
    return (a, b)


def _fit(name: str) -> str:
    return name if len(name) <= 64 else name[:64].rstrip()


def synthetic_kb(n_tickers: int = 2300, seed: int = 20250905) -> Dict[str, Dict[str, Dict[str, tuple]]]:
    """``processed_data`` of a synthetic KB: ~21.5 names per ticker (2300 tickers -> ~50k names)."""
    r = random.Random(seed)
    used_tickers: set = set()
    used_brands: set = set()
    kb: Dict[str, Dict[str, Dict[str, tuple]]] = {}
    for _ in range(n_tickers):
        sym = _ticker_symbol(r, used_tickers)
        while True:
            brand = _word(r)
            if brand not in used_brands:
                used_brands.add(brand)
                break
        attrs: Dict[str, Dict[str, tuple]] = {a: {} for a in ATTRS}

        def add(attr, name):
            name = _fit(name)
            if name and name not in attrs[attr]:
                attrs[attr][name] = _period(r)

        add('id_label', f"{brand} {r.choice(_CO_SUFFIX)}" if r.random() < 0.7 else f"{brand} {_word(r)}")
        add('ticker', sym)
        add('aliases', brand)
        add('aliases', f"{brand} {r.choice(_CO_SUFFIX)}")
        add('aliases', f"{brand}, Inc." if r.random() < 0.5 else f"{brand} {_word(r)} {r.choice(_CO_SUFFIX)}")
        if r.random() < 0.6:
            add('aliases', brand.upper())
        if r.random() < 0.3:
            add('aliases', f"The {brand} Company")
        for _ in range(r.randint(3, 6)):
            k = r.random()
            if k < 0.35:
                add('products', f"{brand} {r.choice(_P_SUFFIX)}")
            elif k < 0.60:
                add('products', _word(r))
            elif k < 0.72:
                add('products', f"{_word(r).lower()}.com")
            elif k < 0.78:
                add('products', f"{brand}+" if r.random() < 0.5 else f"{brand}+ {r.choice(_P_SUFFIX)}")
            elif k < 0.82:
                add('products', _word(r).lower())            # lowercase alpha: never matches
            elif k < 0.86:
                add('products', f"{_word(r)}{r.randint(2, 99)}")
            else:
                add('products', f"{_word(r)} {_word(r)} {r.choice(_P_SUFFIX)}")
        for _ in range(r.randint(2, 4)):
            k = r.random()
            if k < 0.45:
                add('subsidiaries', f"{brand} {r.choice(_REGION)}")
            elif k < 0.85:
                add('subsidiaries', f"{_word(r)} {r.choice(_CO_SUFFIX)}")
            elif k < 0.95:
                add('subsidiaries', f"{brand} {r.choice(_REGION)} {r.choice(_CO_SUFFIX)}")
            else:
                add('subsidiaries', f"{brand} Software({r.choice(_REGION)})Co.,Ltd.")
        for _ in range(r.randint(1, 3)):
            k = r.random()
            add('owned_entities', f"{_word(r)} {_word(r)}" if k < 0.5 else f"{brand} {_word(r)} {r.choice(_UNIT)}")
        for _ in range(r.randint(1, 2)):
            add('ceos', _person(r))
        for _ in range(r.randint(4, 8)):
            add('board_members', _person(r))
        kb[sym] = attrs
    return kb
