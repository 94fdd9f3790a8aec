"""CPU checks of the stationary kernel's LDS layouts (bcfft_stat.hip): every access pattern is
bank-conflict free under the MI355X LDS lane-group model (tools/lds_banks.py), and the
closed-form address shortcuts in the kernel equal the layout functions they replace."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import lds_banks as M  # noqa: E402


@pytest.mark.parametrize("b,es", [(128, 4), (128, 2), (64, 4), (64, 2)])
def test_y_image_and_staging_conflict_free(b, es):
    pi, cols = M.KNOWN[(b, es)]
    w = M.check(M.geo(b, es), pi, cols)
    assert max(w.values()) == 1, w


@pytest.mark.parametrize("b,ni", [(128, 32), (64, 32), (64, 64)])
def test_a_slots_conflict_free(b, ni):
    G = M.ageo(b, ni)
    ns = 4 * ni // G["RPWF"]
    tsw = [s // (ns // 2) for s in range(ns)]             # the kernel's tsw: top bit of the slot
    assert M.a_writes(G, tsw) == 1
    assert M.a_reads(G, tsw) == 1


def _swz(L, es, r):
    return (2 * (r & 7) if L == 4 else (r & 15)) if es == 4 else (r & 7)


@pytest.mark.parametrize("b,es", [(128, 4), (128, 2), (64, 4), (64, 2)])
def test_dma_offsets_closed_form(b, es):
    """dma_tile: byte ^ (swz(row) << 4) == vb[q % DP] + q KiB (q KiB goes in soffset)."""
    L = 4 if b == 128 else 2
    rb = b * es
    ndma = (64 // L) * rb // 1024
    rpk = 1024 // rb
    dp = min(16 // rpk, ndma)
    for wave in range(8):
        for dl in range(64):
            for q in range(ndma):
                byte = (wave * ndma + q) * 1024 + dl * 16
                vb = wave * ndma * 1024 + ((dl * 16) ^ (_swz(L, es, (q % dp) * rpk + dl * 16 // rb) << 4))
                assert byte ^ (_swz(L, es, byte // rb) << 4) == vb + q * 1024


@pytest.mark.parametrize("b,nq,sa,nwf", [(128, 4, 1, 8), (64, 8, 2, 4), (64, 8, 2, 8)])
def test_a_unit_bases(b, nq, sa, nwf):
    """forward's split writes and cmac's reads: aunit(f, prec, lq, s) == lane base + bin offset."""
    L = 4 if b == 128 else 2
    for s in range(nwf):
        tsw = s // (nwf // 2)
        for f in range(b // 2):
            k1, k2 = f >> 4, f & 15
            for prec in range(2):
                for lq in range((64 // L) // 4):
                    a = 16 * ((f * 2 * nq + prec * nq + lq) ^ (((f >> 4) ^ tsw) << sa))
                    ax = (k1 ^ tsw) << sa
                    assert a == 16 * ((prec * nq + lq) ^ ax) + k1 * 16 * 32 * nq + k2 * 16 * 2 * nq
