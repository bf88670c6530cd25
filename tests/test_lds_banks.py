"""Exhaustive bank-conflict check of the conv3x3 LDS window layout (hn_hardnet.hip).

ds_read_b128 on gfx950 serves a wave in four 16-lane groups (MI355X_MICROARCH.md, LDS):
{0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}; a
group is conflict-free when its 16 addresses fall in 16 distinct 16-byte slots of the
256-byte bank row.  This mirrors the kernel's address arithmetic for every conv config,
tap and M tile and asserts conflict-freedom."""
import pytest

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]

# (CIN, COUT, HIN, S, NP, TR, WM, WN) -- the HN_CONV instantiations
CONFIGS = {
    "1": (32, 32, 32, 1, 1, 8, 4, 1),
    "1v1": (32, 32, 32, 1, 1, 4, 4, 1),
    "2": (32, 64, 32, 2, 1, 8, 2, 2),
    "2v1": (32, 64, 32, 2, 1, 4, 2, 2),
    "3": (64, 64, 16, 1, 1, 16, 2, 2),
    "3v1": (64, 64, 16, 1, 1, 8, 2, 2),
    "4": (64, 128, 16, 2, 1, 8, 1, 4),
    "4v1": (64, 128, 16, 2, 1, 4, 1, 4),
    "5": (128, 128, 8, 1, 2, 8, 1, 4),
    "5v1": (128, 128, 8, 1, 1, 8, 1, 4),
    "2t2": (32, 64, 32, 2, 1, 2, 1, 2),
}


def row_stride(ncols, wout, s):
    rs = ncols * 80
    if wout >= 32:
        return rs
    want = 0 if wout == 16 else 8
    while (s * rs // 16) % 16 != want:
        rs += 16
    return rs


def geometry(cin, cout, hin, s, np_, tr, wm, wn):
    hout = hin // s
    rin = tr + 2 if s == 1 else 2 * tr + 1
    ncols = hin + 2 if s == 1 else hin + 1
    half = (ncols + 1) // 2
    rs = row_stride(ncols, hout, s)
    ps = rin * rs
    bm = np_ * tr * hout
    mt = bm // wm // 32
    return dict(hout=hout, rin=rin, ncols=ncols, half=half, rs=rs, ps=ps, bm=bm, mt=mt,
                lds=2 * np_ * ps)


@pytest.mark.parametrize("layer", sorted(CONFIGS))
def test_conv_window_reads_conflict_free(layer):
    cin, cout, hin, s, np_, tr, wm, wn = CONFIGS[layer]
    g = geometry(*CONFIGS[layer])
    wout = g["hout"]

    def colofs(kx):
        return kx if s == 1 else (g["half"] + (kx >> 1) if kx & 1 else kx >> 1)

    for w in range(wm):
        for mt in range(g["mt"]):
            base = []
            for lane in range(64):
                r, h = lane & 31, lane >> 5
                m = (w * g["mt"] + mt) * 32 + r
                npi, rem = divmod(m, tr * wout)
                yl, xo = divmod(rem, wout)
                base.append(npi * g["ps"] + yl * s * g["rs"] + xo * 80 + h * 16)
            for tap in range(9):
                ky, kx = divmod(tap, 3)
                for ks in range(2):
                    toff = ky * g["rs"] + colofs(kx) * 80 + ks * 32
                    for grp in GROUPS:
                        addrs = [base[l] + toff for l in grp]
                        assert all(a % 16 == 0 for a in addrs)
                        slots = {(a // 16) % 16 for a in addrs}
                        assert len(slots) == 16, (layer, w, mt, tap, ks, grp[0])


@pytest.mark.parametrize("layer", sorted(CONFIGS))
def test_conv_lds_fits(layer):
    g = geometry(*CONFIGS[layer])
    assert g["lds"] <= 160 * 1024
    cin, cout = CONFIGS[layer][0], CONFIGS[layer][1]
    assert cin % 32 == 0 and cout % (32 * CONFIGS[layer][7]) == 0


def _front_dw_lane_map():
    src = open(__file__.replace("tests/test_lds_banks.py", "hardnetnas_amd/csrc/hn_front.hip")).read()
    body = src[src.index("kDwLane[64] = {") + len("kDwLane[64] = {"):]
    return [int(v) for v in body[:body.index("}")].replace("\n", " ").split(",") if v.strip()]


def test_front_dw_lane_map():
    """hn_front.hip dw / maxpool window reads: lane -> (ox, q) table is a bijection onto the
    8x8 (pixel, channel-quad) block and every ds_read_b128 16-lane group hits 16 distinct
    16-byte slots for all kx taps (pixel stride PS = 36 floats, stride-2 columns)."""
    tab = _front_dw_lane_map()
    assert sorted(tab) == list(range(64))
    for g in GROUPS:
        for base_ox in (0, 8):
            for dx in range(5):
                slots = set()
                for lane in g:
                    ox, q = base_ox + (tab[lane] >> 3), tab[lane] & 7
                    byte = ((2 * ox + dx) * 36 + 4 * q) * 4
                    slots.add((byte // 16) % 16)
                assert len(slots) == 16, (g, dx)


def test_front_pw_epilogue_writes_conflict_free():
    """MFMA epilogue (pw and the maxpool stem path): lane (px = l & 31, h) writes float4
    2q + h of pixel px at PS = 36 floats -- conflict-free for every q."""
    for g in GROUPS:
        for q in range(4):
            slots = {(((lane & 31) * 36 + 4 * (2 * q + (lane >> 5))) * 4 // 16) % 16 for lane in g}
            assert len(slots) == 16


@pytest.mark.parametrize("hin,s", [(16, 1), (16, 2), (8, 1), (8, 2), (4, 1)])
def test_irf_dw_window_reads_conflict_free(hin, s):
    """hn_irf.hip dw window reads: lane -> (run, quad) = ((l >> 2) & 7, (l & 3) | (l >> 5) << 2),
    run = R output pixels of one row (R = 4 at stride 1, 2 at stride 2), pixel stride 36
    floats; every ds_read_b128 group hits 16 distinct 16-byte slots for every window column
    (8x8 at stride 2, where a run spans a quarter of an input row pair: at most 2-way)."""
    r = 4 if s == 1 else 2
    hout = hin // s
    for it0 in range(0, 512, 64):
        for c in range(8):  # window column
            for g in GROUPS:
                slots = set()
                for lane in g:
                    q = (lane & 3) | ((lane >> 5) << 2)
                    run = (it0 >> 6) * 8 + ((lane >> 2) & 7)
                    o0 = run * r
                    pl, oy, ox0 = o0 // (hout * hout), (o0 // hout) % hout, o0 % hout
                    pix = (pl * hin + oy * s) * hin + ox0 * s + c
                    slots.add(((pix * 36 + 4 * q) * 4 // 16) % 16)
                assert len(slots) >= (8 if (hin, s) == (8, 2) else 16)


@pytest.mark.parametrize("kk", [3, 5])
def test_front_irf_dw_reads_conflict_free(kk):
    """hn_front.hip IRF-form dw window reads: wave w, lane (px = l & 31, h = l >> 5) reads band
    pixel p = 32 (w & 1) + px (output row p >> 4, column ox = p & 15), channels
    16 (w >> 1) + 8 h (+4), at padded input column 2 ox + dx of ring row
    2 (r0 + row) - PAD + dy.  Columns are split even / odd (position c / 2 or HALF + c / 2),
    pixel stride 36 floats, row stride RS = PC * 36 rounded up to 64 floats: every
    ds_read_b128 group hits 16 distinct 16-byte slots for every band, dy and dx."""
    pad, rb = kk // 2, 4
    ir = 2 * (rb - 1) + kk
    pc = 32 + 2 * pad
    half = (pc + 1) // 2
    rs = (pc * 36 + 63) // 64 * 64
    assert half + pc // 2 <= rs // 36  # positions fit the row
    for w in range(4):
        for band in range(4):
            r0 = band * rb
            for dy in range(kk):
                for dx in range(kk):
                    for j in range(2):
                        for g in GROUPS:
                            slots = set()
                            for lane in g:
                                px, h = lane & 31, lane >> 5
                                p = 32 * (w & 1) + px
                                orr, ox = p >> 4, p & 15
                                c0 = 16 * (w >> 1) + 8 * h + 4 * j
                                slot = (2 * (r0 + orr) - pad + dy + pad + ir) % ir
                                pos = half + ox + (dx >> 1) if dx & 1 else ox + (dx >> 1)
                                slots.add(((slot * rs + pos * 36 + c0) * 4 // 16) % 16)
                            assert len(slots) == 16, (kk, w, band, dy, dx, g[0])


def _front_nf_maps(pad):
    """hn_front.hip NF lane permutations: pxm (stem / pw MFMA column -> image column) and dwx
    (16x16 pwl column -> output column)."""
    pxm = [2 * (n & 15) + (((n >> 4) & 1) ^ (pad & 1)) for n in range(32)]
    dwx = [2 * n if n < 4 else 2 * (n - 4) + 1 if n < 12 else 2 * (n - 8) for n in range(16)]
    return pxm, dwx


@pytest.mark.parametrize("kk", [3, 5])
def test_front_nf_dw_reads_conflict_free(kk):
    """NF dw window reads: lane l reads output column dwx[l & 15], channels 8 (l >> 4) (+4) at padded
    input column 2 ox + dx of its wave's ring row (even / odd split positions, pixel stride 36
    floats): every ds_read_b128 group hits 16 distinct 16-byte slots.  In column order (ox = l & 15)
    the groups were 2-way conflicted -- the 35 % SQ_LDS_BANK_CONFLICT share of the k5 front."""
    pad = kk // 2
    half = (32 + 2 * pad + 1) // 2
    _, dwx = _front_nf_maps(pad)
    assert sorted(dwx) == list(range(16))
    worst_identity = 0
    for dx in range(kk):
        for j in range(2):
            for perm in (dwx, list(range(16))):
                for g in GROUPS:
                    slots = set()
                    for lane in g:
                        ox = perm[lane & 15]
                        pos = half + ox + (dx >> 1) if dx & 1 else ox + (dx >> 1)
                        slots.add(((pos * 36 + 8 * (lane >> 4) + 4 * j) * 4 // 16) % 16)
                    if perm is dwx:
                        assert len(slots) == 16, (kk, dx, j, g[0])
                    else:
                        worst_identity = max(worst_identity, 16 - len(slots))
    assert worst_identity > 0  # the column-order map this replaced


@pytest.mark.parametrize("kk", [3, 5])
def test_front_nf_pw_writes_conflict_free(kk):
    """NF pw epilogue: lane (n = l & 31, h) writes float4 2q + h of image column pxm[n] at position
    colpos(PAD + pxm[n]) (pixel stride 36 floats); ds_write_b128 serves 8 groups of 8 consecutive
    lanes, conflict-free when their addresses fall in 8 distinct 16-byte slots of 128 bytes."""
    pad = kk // 2
    half = (32 + 2 * pad + 1) // 2
    pxm, _ = _front_nf_maps(pad)
    assert sorted(pxm) == list(range(32))
    for q in range(4):
        for g0 in range(0, 64, 8):
            slots = set()
            for lane in range(g0, g0 + 8):
                c = pad + pxm[lane & 31]
                pos = half + c // 2 if c & 1 else c // 2
                slots.add(((pos * 36 + 4 * (2 * q + (lane >> 5))) * 4 // 16) % 8)
            assert len(slots) == 8, (kk, q, g0)


def test_front_xch_accesses_conflict_free():
    """k5 front XCH form: wave w = channel group w of the band's four rows, lane (row l >> 4, column
    l & 15) reads ring row 2 (r0 + row) - PAD + dy at split position pos(column, dx), channels
    8 w (+4); then writes its hi / lo 16-byte chunk to s_x[plane][row][column][w ^ ((column >> 1) & 3)],
    and wave w reads row w back as lane (column l & 15, channel group l >> 4).  Row stride RS is a
    multiple of 64 floats, so the two rows a read group mixes share one slot pattern."""
    kk, pad, ps = 5, 2, 36
    pc = 32 + 2 * pad
    half, rs, ir = (pc + 1) // 2, (pc * ps + 63) // 64 * 64, 2 * 3 + kk
    for w in range(4):
        for r0 in (0, 4, 8, 12):
            for dy in range(kk):
                for dx in range(kk):
                    for j in range(2):
                        for g in GROUPS:
                            slots = set()
                            for lane in g:
                                rr, ox = lane >> 4, lane & 15
                                slot = (2 * (r0 + rr) - pad + dy + pad + ir) % ir
                                pos = half + ox + (dx >> 1) if dx & 1 else ox + (dx >> 1)
                                slots.add(((slot * rs + pos * ps + 8 * w + 4 * j) * 4 // 16) % 16)
                            assert len(slots) == 16, (w, r0, dy, dx, j, g[0])
        for g0 in range(0, 64, 8):  # ds_write_b128: 8 groups of 8 lanes, slots of 128 bytes
            slots = {((((l >> 4) * 16 + (l & 15)) * 4 + (w ^ (((l & 15) >> 1) & 3))) * 16 // 16) % 8
                     for l in range(g0, g0 + 8)}
            assert len(slots) == 8, (w, g0)
        for g in GROUPS:
            slots = {(((w * 16 + (l & 15)) * 4 + ((l >> 4) ^ (((l & 15) >> 1) & 3))) * 16 // 16) % 16 for l in g}
            assert len(slots) == 16, (w, g[0])


def test_front_x3_swizzle_conflict_free():
    """k3 front XCH form (HN_FRONT_XCH3, SW in hn_front.hip): ring pixels of 32 floats, 16-byte channel
    chunk c of position pos at c ^ swz(pos), swz(pos) = (pos + 3 (pos >> 1)) & 7.  The dw reads (lane
    (row l >> 4, column l & 15), chunks 2 w, 2 w + 1 at position pos(column, dx)) hit 16 distinct slots
    per ds_read_b128 group and the pw epilogue writes (lane (n, h): chunk 2 q + h of image column pxm[n])
    8 distinct slots per 8-lane ds_write_b128 group; without the swizzle both conflict."""
    kk, pad, ps = 3, 1, 32
    pc = 32 + 2 * pad
    half, rs = (pc + 1) // 2, pc * ps
    assert rs % 64 == 0  # the rows a read group mixes share one slot pattern
    pxm, _ = _front_nf_maps(pad)
    for swz, want in ((lambda p: (p + 3 * (p >> 1)) & 7, True), (lambda p: 0, False)):
        ok = True
        for w in range(4):
            for dx in range(kk):
                for j in range(2):
                    for g in GROUPS:
                        slots = set()
                        for lane in g:
                            ox = lane & 15
                            pos = half + ox + (dx >> 1) if dx & 1 else ox + (dx >> 1)
                            slots.add(((pos * ps + 4 * ((2 * w + j) ^ swz(pos))) * 4 // 16) % 16)
                        ok &= len(slots) == 16
        for q in range(4):
            for g0 in range(0, 64, 8):
                slots = set()
                for lane in range(g0, g0 + 8):
                    c = pad + pxm[lane & 31]
                    pos = half + c // 2 if c & 1 else c // 2
                    slots.add(((pos * ps + 4 * ((2 * q + (lane >> 5)) ^ swz(pos))) * 4 // 16) % 8)
                ok &= len(slots) == 8
        assert ok == want


@pytest.mark.parametrize("kk", [3, 5])
def test_front_irf_fold_positions_are_interior(kk):
    """The pwl partial-sum fold uses the 16 interior even positions from 1 and the 16 interior
    odd positions from HALF + PAD - 1: never a zero pad column."""
    pad = kk // 2
    pc = 32 + 2 * pad
    half = (pc + 1) // 2
    pos = {c: (half + c // 2 if c & 1 else c // 2) for c in range(pc)}
    padpos = {pos[c] for c in range(pc) if c < pad or c >= 32 + pad}
    for start in (1, half + pad - 1):
        span = set(range(start, start + 16))
        assert not span & padpos
        assert (start + 15) * 36 + 36 <= (pc * 36 + 63) // 64 * 64 or start + 15 < pc


# 64-byte swizzled window layout of k_conv_ws (hn_hardnet.hip ConvCfg PX = 64, stride 2):
# chunk q (16 B = 8 channels) of window row wr at slot q ^ ((wr // S) & 3), no pixel pad, one
# spare column slot between the even and the odd half
SWZ_CONFIGS = {"4np2": (64, 128, 16, 2, 2, 8, 1, 4), "4": (64, 128, 16, 2, 1, 8, 1, 4),
               "4np2w22": (64, 128, 16, 2, 2, 8, 2, 2),
               "5np4a": (128, 128, 8, 1, 4, 8, 4, 2), "5np4b": (128, 128, 8, 1, 4, 8, 2, 2)}


@pytest.mark.parametrize("layer", sorted(SWZ_CONFIGS))
def test_swizzled_window_reads_and_writes_conflict_free(layer):
    cin, cout, hin, s, np_, tr, wm, wn = SWZ_CONFIGS[layer]
    hout = hin // s
    rin, ncols = (2 * tr + 1, hin + 1) if s == 2 else (tr + 2, hin + 2)
    half = (ncols + 1) // 2 + 1
    rs = (half + ncols // 2) * 64 if s == 2 else ncols * 64
    ps = rin * rs
    mt_n = np_ * tr * hout // wm // 32
    assert 2 * 2 * np_ * ps <= 160 * 1024  # double-buffered hi + lo planes

    def colofs(kx):
        if s == 1:
            return kx
        return half + (kx >> 1) if kx & 1 else kx >> 1

    for w in range(wm):
        for mt in range(mt_n):
            for tap in range(9):
                ky, kx = divmod(tap, 3)
                for ks in range(2):
                    addrs = []
                    for lane in range(64):
                        r, h = lane & 31, lane >> 5
                        m = (w * mt_n + mt) * 32 + r
                        npi, rem = divmod(m, tr * hout)
                        yl, xo = divmod(rem, hout)
                        wr = yl * s + ky
                        q = (2 * ks + h) ^ ((wr // s) & 3)
                        addrs.append(npi * ps + wr * rs + (colofs(kx) + xo) * 64 + 16 * q)
                    for grp in GROUPS:
                        slots = {(addrs[l] // 16) % 16 for l in grp}
                        assert len(slots) == 16, (layer, w, mt, tap, ks, grp[0])
    # producer stores: unit u = (pixel, 8-channel group g); ds_write_b128 lanes in groups of 8
    units = np_ * rin * ncols * 4
    addr = []
    for u in range(units):
        g, pix = u & 3, u >> 2
        wc, t2 = pix % ncols, pix // ncols
        wr, npi = t2 % rin, t2 // rin
        pc = wc if s == 1 else ((wc >> 1) + half if wc & 1 else wc >> 1)
        addr.append(npi * ps + wr * rs + pc * 64 + 16 * (g ^ ((wr // s) & 3)))
    assert len(set(addr)) == units
    for k in range(0, units - 7, 8):
        if (k // 64) != ((k + 7) // 64):
            continue
        slots = {(a // 16) % 16 for a in addr[k:k + 8]}
        assert len(slots) == 8, (layer, k)


def _band_sw(p):  # hn_irf.hip band_sw
    return ((p >> 1) & 1) | (((p >> 4) & 1) << 1) | (((p >> 2) & 1) << 2)


def test_irf_band_buffer_conflict_free():
    """k_irf2's band buffer (IRF_BAND, 128 pixels x 32 floats, chunk c of pixel p at c ^ band_sw(p)):
    the pwl's ds_read_b128 operand reads (lane: pixel 32 t + (l & 31), chunks 4 s + 2 (l >> 5) + k)
    hit 16 distinct 16-byte slots per group, and the dw's ds_write_b128 stores (8-lane groups; lane
    -> run, channel quad as in irf_core) 8 distinct slots of the 128-byte write row."""
    for pt in range(4):
        for s in range(2):
            for k in range(2):
                for g in GROUPS:
                    slots = set()
                    for l in g:
                        p, c = pt * 32 + (l & 31), 4 * s + 2 * (l >> 5) + k
                        slots.add((p * 8 + (c ^ _band_sw(p))) % 16)
                    assert len(slots) == 16, (pt, s, k)
    for band in range(2):
        for w in range(4):
            for r in range(4):
                for g0 in range(0, 64, 8):
                    slots = set()
                    for lane in range(g0, g0 + 8):
                        it = w * 64 + lane + 256 * band
                        q = (lane & 3) | ((lane >> 5) << 2)
                        run = (it >> 6) * 8 + ((lane >> 2) & 7)
                        p = (run * 4 + r) & 127
                        slots.add((q ^ _band_sw(p)) % 8)
                    assert len(slots) == 8, (band, w, r, g0)


def test_irf_weight_pad_slots_conflict_free():
    """IRF_WPAD: dw weight float4 i in the pad slot of s_pw pixel i (byte 144 i + 128); a 16-lane read
    group touches 4 channel quads of one tap (broadcast within a quad): 4 distinct slots."""
    for k in (3, 5):
        for tap in range(k * k):
            for g in GROUPS:
                addrs = {}
                for l in g:
                    q = (l & 3) | ((l >> 5) << 2)
                    a = (tap * 8 + q) * 144 + 128
                    addrs.setdefault((a // 16) % 16, set()).add(a)
                assert all(len(v) == 1 for v in addrs.values()), (k, tap)


# hn_wino1.hip (1-D Winograd F(2,3)): (CIN, COUT, H, NP, WM, WN) of conv3 / conv5; whole patches per
# work tile, the image holds each patch's H rows and one zero row that the padding rows read
W1_CONFIGS = {"3": (64, 64, 16, 1, 2, 2), "5": (128, 128, 8, 2, 1, 4)}
WRITE_GROUPS = [list(range(i, i + 8)) for i in range(0, 64, 8)]  # ds_write_b128: 8 x 8 contiguous


def w1_geometry(cin, cout, h, np_, wm, wn):
    ntx = h // 2
    xrow = ntx * 64
    rs = 4 * xrow
    ps = h * rs
    bm = np_ * h * ntx
    return dict(ntx=ntx, tr=h, xrow=xrow, rs=rs, ps=ps, zrow=np_ * ps, mt=bm // wm // 32, units=np_ * h * ntx * 4)


@pytest.mark.parametrize("layer", sorted(W1_CONFIGS))
def test_wino1_operand_reads_conflict_free(layer):
    """Every 32x32x16 operand read of k_conv_w1 (lane: M index r = (row, column pair), channel half
    h; chunk 2 ks + h of window row wr = yl + ky at chunk ^ (wr & 3); window rows 0 and H + 1 are
    the zero row)."""
    cin, cout, h, np_, wm, wn = W1_CONFIGS[layer]
    g = w1_geometry(*W1_CONFIGS[layer])
    for w in range(wm):
        for mt in range(g["mt"]):
            for kx in range(24):
                xi, ky, ks = kx // 6, (kx % 6) // 2, kx % 2
                addrs = []
                for lane in range(64):
                    r, hh = lane & 31, lane >> 5
                    m = (w * g["mt"] + mt) * 32 + r
                    npi, rem = divmod(m, g["tr"] * g["ntx"])
                    yl, t = divmod(rem, g["ntx"])
                    wr = yl + ky
                    rowb = npi * g["ps"] + (wr - 1) * g["rs"] if 1 <= wr <= g["tr"] else g["zrow"]
                    addrs.append(rowb + t * 64 + 16 * ((2 * ks + hh) ^ (wr & 3)) + xi * g["xrow"])
                for grp in GROUPS:
                    slots = {(addrs[l] // 16) % 16 for l in grp}
                    zero = {addrs[l] for l in grp if addrs[l] >= g["zrow"]}
                    # lanes of the zero row may share an address (broadcast); distinct addresses need distinct slots
                    distinct = {a for a in (addrs[l] for l in grp)}
                    assert len({(a // 16) % 16 for a in distinct}) == len(distinct), (layer, w, mt, kx, grp[0], len(zero))


@pytest.mark.parametrize("layer", sorted(W1_CONFIGS))
def test_wino1_producer_writes_conflict_free(layer):
    """The producers' ds_write_b128 of one transform position xi: unit u = ((patch, row y), column
    pair, 8-channel group) -> chunk g ^ ((y + 1) & 3) of position t; each 8-lane group covers 128
    distinct contiguous bytes."""
    g = w1_geometry(*W1_CONFIGS[layer])
    for k in range(-(-g["units"] // 256)):
        for wave in range(4):
            for xi in range(4):
                addrs = []
                for lane in range(64):
                    u = wave * 64 + lane + k * 256
                    gg, t, rest = u & 3, (u >> 2) % g["ntx"], (u >> 2) // g["ntx"]
                    y, npi = rest % g["tr"], rest // g["tr"]
                    addrs.append(npi * g["ps"] + y * g["rs"] + xi * g["xrow"] + t * 64 + 16 * (gg ^ ((y + 1) & 3)))
                for grp in WRITE_GROUPS:
                    slots = {(addrs[l] // 16) % 16 for l in grp}
                    assert len(slots) == 8, (layer, k, wave, xi, grp[0])


# hn_wino1.hip k_conv_w4 (conv3 as F(4,3)): (CIN, COUT, H, NP, WN); image [patch][xi][row -1 .. H][quad]
# [32 channels bf16], 256-byte rows, chunk c of input row r at c ^ 2 (r & 1)
W4_CONFIGS = {"3": (64, 64, 16, 1, 4)}


def w4_geometry(cin, cout, h, np_, wn):
    ntx = h // 4
    rb = ntx * 64
    xb = (h + 2) * rb
    return dict(ntx=ntx, h=h, rb=rb, xb=xb, mt=np_ * h * ntx // 16, units=np_ * h * ntx * 4)


def w4_xi(xo):
    return 0 if xo == 0 else 5 if xo == 1 else xo - 1


@pytest.mark.parametrize("layer", sorted(W4_CONFIGS))
def test_wino4_operand_reads_conflict_free(layer):
    """Every 16x16x32 B-operand read of k_conv_w4 (lane: position l & 15 of M tile mt, 16-byte chunk
    l >> 4; input row r = y + ky - 1, rows -1 / H being the (patch, xi) block's zero rows)."""
    g = w4_geometry(*W4_CONFIGS[layer])
    for mt in range(g["mt"]):
        for kx in range(18):
            xi, ky = w4_xi(kx // 3), kx % 3
            for plane in range(2):
                addrs = []
                for lane in range(64):
                    pos = mt * 16 + (lane & 15)
                    npi, rem = divmod(pos, g["h"] * g["ntx"])
                    y, t = divmod(rem, g["ntx"])
                    r = y + ky - 1
                    addrs.append(plane * 10 ** 6 + (npi * 6 + xi) * g["xb"] + (r + 1) * g["rb"] + t * 64
                                 + 16 * ((lane >> 4) ^ (2 * (r & 1))))
                for grp in GROUPS:
                    distinct = {addrs[l] for l in grp}
                    assert len(distinct) == 16
                    assert len({(a // 16) % 16 for a in distinct}) == 16, (layer, mt, kx, grp[0])


@pytest.mark.parametrize("layer", sorted(W4_CONFIGS))
def test_wino4_producer_writes_conflict_free(layer):
    """The producers' ds_write_b128 of one xi: unit u = (patch, row y, quad t, 8-channel group g) ->
    chunk g ^ 2 (y & 1) of position t of row y; each 8-lane group covers 128 distinct bytes."""
    g = w4_geometry(*W4_CONFIGS[layer])
    for k in range(g["units"] // 256):
        for wave in range(4):
            for xi in range(6):
                addrs = []
                for lane in range(64):
                    u = wave * 64 + lane + k * 256
                    gg, t, rest = u & 3, (u >> 2) % g["ntx"], (u >> 2) // g["ntx"]
                    y, npi = rest % g["h"], rest // g["h"]
                    addrs.append((npi * 6 + xi) * g["xb"] + (y + 1) * g["rb"] + t * 64 + 16 * (gg ^ (2 * (y & 1))))
                for grp in WRITE_GROUPS:
                    assert len({(addrs[l] // 16) % 16 for l in grp}) == 8, (layer, k, wave, xi, grp[0])


# ---- k_c12w (hn_c12w.hip): conv1 as a 1-D Winograd F(4,3) inside the fused stem+conv1+conv2 kernel ----
C12W_VROW = 6 * 8 * 128  # W0 ring bytes per a0 row: V records (xi, tile T), 128 B, chunk c at c ^ T


def test_c12w_conv1_operand_reads_conflict_free():
    """P2's ds_read_b128 of V_xi (lane n = T + 8 j: tile T of a0 row y0 + j - 1 + ky; K-group g16 = hi chunk
    g16 / lo chunk 4 + g16) for every ring slot pair, ky and xi."""
    for slot0 in range(6):
        for ky in range(3):
            for xi in range(6):
                for plane in range(2):
                    addrs = []
                    for lane in range(64):
                        n, g16 = lane & 15, lane >> 4
                        t, j = n & 7, n >> 3
                        slot = (slot0 + j + ky) % 6
                        c = g16 + 4 * plane
                        addrs.append(slot * C12W_VROW + (xi * 8 + t) * 128 + 16 * (c ^ t))
                    for grp in GROUPS:
                        assert len({(addrs[l] // 16) % 16 for l in grp}) == 16, (slot0, ky, xi, plane, grp[0])


def test_c12w_transform_writes_conflict_free():
    """P1's ds_write_b128 of the V records after the hi / lo swap: lane (tile T = l & 7, row j = (l >> 3) & 1,
    K-group g16) of channel half ph writes chunk (2 ph + g16 / 2 + 4 (g16 & 1)) ^ T; each 8-lane group
    covers 8 distinct 16-byte slots of a 128-byte bank row."""
    for ph in range(2):
        for y0 in range(6):
            for xi in range(6):
                addrs = []
                for lane in range(64):
                    t, j, g16 = lane & 7, (lane >> 3) & 1, lane >> 4
                    c = (2 * ph + (g16 >> 1) + 4 * (g16 & 1)) ^ t
                    addrs.append(((y0 + j + 1) % 6) * C12W_VROW + (xi * 8 + t) * 128 + 16 * c)
                for grp in WRITE_GROUPS:
                    assert len({(addrs[l] // 16) % 8 for l in grp}) == 8, (ph, y0, xi, grp[0])


def test_c12w_records_cover_each_chunk_once():
    """Over the 4 P1 waves' channel halves and both swap parities, every (record, chunk) of a V row is written
    exactly once, and P2 reads exactly the chunk holding its K-group's 8 channels (hi and lo)."""
    seen = {}
    for ph in range(2):
        for lane in range(64):
            t, g16 = lane & 7, lane >> 4
            ch0 = 16 * ph + 4 * (g16 & ~1)  # the 8 channels this lane holds after the swap
            plane = g16 & 1
            c = (2 * ph + (g16 >> 1) + 4 * plane)
            key = (t, c ^ t)
            seen.setdefault(key, set()).add((ch0, plane, (lane >> 3) & 1))
    for t in range(8):
        for g in range(4):  # P2: K-group g = channels 8 g .. 8 g + 7
            for plane in range(2):
                got = seen[(t, (g + 4 * plane) ^ t)]
                assert {(c, p) for c, p, _ in got} == {(8 * g, plane)}



# ---- k_c12s (hn_c12w.hip): P2's N index = tile n >> 1 of row n & 1, W0 rows padded to VROW + 128, W1 ring of 10 ----
C12S_VROW = C12W_VROW + 128
C12S_W1ROW = 33 * 160


def _w1_slot(x):  # even (x + 1) -> (x + 1) / 2, odd -> 17 + x / 2
    return 17 + (x >> 1) if (x + 1) & 1 else (x + 1) >> 1


def test_c12s_conv1_operand_reads_conflict_free():
    """P2's ds_read_b128 of V_xi in k_c12s (lane n = 2 tt + tj: tile tt of a0 row 4 band + 2 rp + tj - 1 + ky,
    ring slot (32 p + r) % 10, rows -1 / 32 -> the zero row 10): conflict-free for every real row pair; only a
    pair that includes the zero row may collide (2 of 8 bands, one ky)."""
    for p in range(10):
        for band in range(8):
            for rp in range(2):
                for ky in range(3):
                    for xi in range(6):
                        for plane in range(2):
                            addrs, pad = [], False
                            for lane in range(64):
                                n, g16 = lane & 15, lane >> 4
                                tt, tj = n >> 1, n & 1
                                r = 4 * band + 2 * rp + tj - 1 + ky
                                pad |= not 0 <= r <= 31
                                slot = 10 if not 0 <= r <= 31 else (32 * p + r) % 10
                                addrs.append(slot * C12S_VROW + xi * 1024 + tt * 128 + 16 * ((g16 + 4 * plane) ^ tt))
                            if pad:
                                continue
                            for grp in GROUPS:
                                assert len({(addrs[l] // 16) % 16 for l in grp}) == 16, (p, band, rp, ky, xi, plane)


def test_c12s_p2_epilogue_writes_two_way_at_most():
    """P2's epilogue ds_write_b128 into W1 (160-byte pixels, column 4 tt + i of a1 row (32 p + 4 band + 2 rp + tj)
    % 10, the 16-byte chunk 32 g1 + 16 (g16 / 2) + 64 (g16 & 1)): each 8-lane group holds 4 tiles x 2 rows on at
    least 4 distinct 16-byte positions (k_c12w's mapping: 2 positions, 4-way) -- including the ring's wrap."""
    for p in range(10):
        for band in range(8):
            for rp in range(2):
                for g1 in range(2):
                    for i in range(4):
                        addrs = []
                        for lane in range(64):
                            n, g16 = lane & 15, lane >> 4
                            tt, tj = n >> 1, n & 1
                            row = (32 * p + 4 * band + 2 * rp + tj) % 10
                            addrs.append(row * C12S_W1ROW + _w1_slot(4 * tt + i) * 160 + 32 * g1 + 16 * (g16 >> 1)
                                         + 64 * (g16 & 1))
                        for grp in WRITE_GROUPS:
                            pos = [(addrs[l] // 16) % 8 for l in grp]
                            assert max(pos.count(v) for v in pos) <= 2, (p, band, rp, g1, i, grp[0])


def test_c12s_p1_writes_conflict_free_on_padded_rows():
    """P1's V-record stores (k_c12w's lane map) stay conflict-free with the padded W0 row stride."""
    for ph in range(2):
        for y0 in range(10):
            for xi in range(6):
                addrs = []
                for lane in range(64):
                    t, j, g16 = lane & 7, (lane >> 3) & 1, lane >> 4
                    c = (2 * ph + (g16 >> 1) + 4 * (g16 & 1)) ^ t
                    addrs.append(((y0 + j) % 10) * C12S_VROW + (xi * 8 + t) * 128 + 16 * c)
                for grp in WRITE_GROUPS:
                    assert len({(addrs[l] // 16) % 8 for l in grp}) == 8, (ph, y0, xi, grp[0])
