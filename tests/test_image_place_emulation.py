"""CPU emulation of the fused CM -> image write-out's index math (csrc/common_mode.hip, cm_place):
every thread of a 256-thread workgroup walks its (run, full chunk) items incrementally (row-run
panels; column-run panels: the line-aligned walk, PR_CM_PLACE_LA, or the round-5 4-chunk walk), then
the ragged run ends; the emulation applies the same arithmetic to every tile of the production
epix10k2M geometry (and the small test detectors) and checks that each panel pixel is written
exactly once, at the image element the geometry assigns it, that full chunks are 16-B aligned, and
that every streaming (whole-line) store of the line-aligned walk shares its store instruction with
the other 7 chunks of its 128-B line (a split line is what made streaming stores lose).
The GPU tests check the same end to end (tests/test_kernels_gpu.py::test_image_mode_matches_scatter,
tests/test_production_shapes_gpu.py); this one pins the arithmetic without a GPU."""
import numpy as np
import pytest

from psana_ray_amd.models import get_detector, list_detectors
from psana_ray_amd.models.geometry import make_geometry


def _place_tile(writes, P, R, C, desc, y0, x0, nb=256, la=True):
    """Transcription of cm_place: (image element, tile row, tile col, full chunk, instruction id)
    per element written; the instruction id is (wave, iteration) of the line-aligned walk."""
    b, sy, sx = (int(v) for v in desc)
    b0 = b + y0 * sy + x0 * sx
    rows = sx in (1, -1)
    ln = C if rows else R
    nruns = R if rows else C
    step = sx if rows else sy
    outer = sy if rows else sx
    out = []
    if outer & 3:
        for e in range(R * C):
            a, t = divmod(e, ln)
            r, c = (a, t) if rows else (t, a)
            out.append((b0 + r * sy + c * sx, r, c, False, None))
        return out
    lo = b0 if step > 0 else b0 - (ln - 1)
    head = lo & 3
    ch_lo = (head + 3) >> 2
    nfull = max(0, ((ln + head) >> 2) - ch_lo)
    t_lo = 4 * ch_lo - head if nfull > 0 else ln
    t_hi = t_lo + 4 * nfull if nfull > 0 else ln

    def tile_rc(run, t):
        i = t if step > 0 else ln - 1 - t
        return (run, i) if rows else (i, run)

    if nfull > 0 and not rows and la:
        ob = (lo & ~3) + 4 * ch_lo
        nrg, ng, nw = (nruns + 7) >> 3, (nfull + 14) >> 3, nb // 64
        for wave in range(nw):
            for u in range(wave, nrg * ng, nw):
                rg, g = divmod(u, ng)
                for lane in range(64):
                    ro, j = lane >> 3, lane & 7
                    run = 8 * rg + ro
                    a0 = ob + run * outer
                    k = 8 * g - ((a0 >> 2) & 7) + j
                    if run < nruns and 0 <= k < nfull:
                        base = a0 + 4 * k
                        assert base % 4 == 0
                        for q in range(4):
                            r, c = tile_rc(run, t_lo + 4 * k + q)
                            out.append((base + q, r, c, True, (wave, u)))
    elif nfull > 0:
        span = nfull if rows else ((nfull + 3) >> 2) * 4
        per = nfull if rows else 4 * nruns
        da, dw = nb // per, nb - (nb // per) * per
        outer_n = nruns if rows else (span >> 2)
        for tid in range(nb):
            a, w = divmod(tid, per)
            while a < outer_n:
                run = a if rows else (w >> 2)
                k = w if rows else 4 * a + (w & 3)
                if k < nfull:
                    base = (lo & ~3) + run * outer + 4 * (ch_lo + k)
                    assert base % 4 == 0
                    # the lean form (PR_CM_PLACE2): linear in (run, chunk), signed tile stride
                    ob = (lo & ~3) + 4 * ch_lo
                    assert ob + run * outer + 4 * k == base
                    t0 = t_lo + 4 * k
                    i_lean = (t_lo if step > 0 else ln - 1 - t_lo) + 4 * k * (1 if step > 0 else -1)
                    assert i_lean == (t0 if step > 0 else ln - 1 - t0)
                    for q in range(4):
                        r, c = tile_rc(run, t_lo + 4 * k + q)
                        out.append((base + q, r, c, True, None))
                a += da
                w += dw
                if w >= per:
                    w -= per
                    a += 1
    n_head, n_rag = t_lo, t_lo + (ln - t_hi)
    for e in range(nruns * n_rag):
        run, j = divmod(e, n_rag)
        t = j if j < n_head else t_hi + (j - n_head)
        r, c = tile_rc(run, t)
        out.append((lo + run * outer + t, r, c, False, None))
    return out


@pytest.mark.parametrize("la", [True, False])
@pytest.mark.parametrize("det", ["epix10k2M"] + [d for d in list_detectors() if d.startswith("tiny")])
def test_cm_place_index_math(det, la):
    spec = get_detector(det)
    geo = make_geometry(spec)
    place = geo.panel_placement()
    if place is None:
        pytest.skip("no integer placement for this geometry")
    place = place.reshape(-1, 3)
    imap = geo.index_map().ravel()
    Pn, H, W = spec.frame_shape
    R = spec.asic_rows
    C = 48 if (spec.kind == "epix10ka" and R == 176) else spec.asic_cols   # the production stripe width
    hits = np.zeros(imap.size, np.int32)
    for p in range(Pn):
        for ar in range(H // R):
            for ac in range(W // C):
                writes = _place_tile(hits, 0, R, C, place[p], ar * R, ac * C, la=la)
                for addr, r, c, _full, _ins in writes:
                    hits[addr] += 1
                    assert imap[addr] == p * H * W + (ar * R + r) * W + (ac * C + c)
                # st_img4's streaming test: a chunk whose 128-B line lies inside its run; in the
                # line-aligned walk all 8 chunks of such a line come from one store instruction
                lines = {}
                for addr, _r, _c, full, ins in writes:
                    if full and ins is not None and addr % 4 == 0:
                        lines.setdefault(addr >> 5, set()).add(ins)
                for ln_, ins in lines.items():
                    assert len(ins) == 1, (p, ar, ac, ln_, ins)
    assert np.array_equal(hits, (imap >= 0).astype(np.int32))
