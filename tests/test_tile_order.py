"""CPU checks of the host-side tile tables of the grouped ASPP GEMM."""


def test_grouped_tile_order_cpu():
    """Every tile of every conv appears once, heaviest (most live taps) first."""
    from semantic_segmentation_server_amd.ops import hip_ops as K
    convs = [dict(B=2, OH=33, OW=33, k=1, dil=1, Cin=320, Cout=256)] + [
        dict(B=2, OH=33, OW=33, k=3, dil=r, Cin=320, Cout=256, perm=K.tap_group_perm(2, 33, 33, 3, r, 128))
        for r in (6, 12, 18)]
    o = K.grouped_tile_order(convs, 5).tolist()
    assert len(o) == len(set(o))
    for gi, c in enumerate(convs):
        M = c["perm"].numel() if "perm" in c else 2 * 33 * 33
        assert sorted(v & 0xFFFFFF for v in o if v >> 24 == gi) == list(range(-(-M // 128)))
    assert o[0] >> 24 == 1 and o[-1] >> 24 in (0, 3)  # a full 9-tap rate-6 tile leads



def test_grouped_tile_order_xcd_local_cpu():
    """XCD-local order: a permutation of the LPT table; block i's tile (i % 8 = XCD) comes
    from that XCD's contiguous run of row tiles while the runs last."""
    from semantic_segmentation_server_amd.ops import hip_ops as K
    convs = [dict(B=4, OH=33, OW=33, k=1, dil=1, Cin=320, Cout=256)] + [
        dict(B=4, OH=33, OW=33, k=3, dil=r, Cin=320, Cout=256, perm=K.tap_group_perm(4, 33, 33, 3, r, 128))
        for r in (6, 12)]
    a = K.grouped_tile_order(convs, 5).tolist()
    b = K.grouped_tile_order(convs, 5, xcds=8).tolist()
    assert sorted(a) == sorted(b) and len(set(b)) == len(b)
    n0 = -(-4 * 33 * 33 // 128)  # 1x1 conv's row tiles
    first = [v & 0xFFFFFF for v in b[:8 * 3] if v >> 24 == 0]
    assert all(0 <= t < n0 for t in first)


def test_grouped_tile_order_branch_affine_cpu():
    """Branch-affine order: a permutation of the LPT table in which, while the per-XCD runs
    last, every XCD (block i -> XCD i % 8) sees tiles of a single conv, and every conv gets
    at least one XCD."""
    from semantic_segmentation_server_amd.ops import hip_ops as K
    convs = [dict(B=32, OH=33, OW=33, k=1, dil=1, Cin=320, Cout=256)] + [
        dict(B=32, OH=33, OW=33, k=3, dil=r, Cin=320, Cout=256,
             perm=K.tap_group_perm(32, 33, 33, 3, r, 256)) for r in (6, 12, 18)]
    a = K.grouped_tile_order(convs, 8).tolist()
    b = K.grouped_tile_order_branch(convs, 8).tolist()
    assert sorted(a) == sorted(b) and len(set(b)) == len(b)
    import collections
    seen = {}
    for i, v in enumerate(b):
        if v >> 24:  # 3x3 branches: (almost) one per XCD
            seen.setdefault(i % 8, collections.Counter())[v >> 24] += 1
    for c in seen.values():
        assert c.most_common(1)[0][1] >= 0.9 * sum(c.values())
    assert {c.most_common(1)[0][0] for c in seen.values()} == {1, 2, 3}
    counts = [len(b[x::8]) for x in range(8)]  # equal block counts per XCD
    assert max(counts) - min(counts) <= 1


def test_grouped_tile_order_i8_cpu():
    """int8 grouped ASPP order: every tile of every branch exactly once, heaviest (most live
    taps x K chunks) first; the tap-class permutation leaves whole tiles with fewer taps."""
    import torch
    from semantic_segmentation_server_amd.ops import hip_ops as K
    B, H, C, A = 2, 65, 2048, 256
    convs = [dict(B=B, OH=H, OW=H, Cin=C, Cout=A, k=1)]
    for d in (6, 12, 18):
        convs.append(dict(B=B, OH=H, OW=H, Cin=C, Cout=A, k=3, dil=d,
                          perm=K.tap_group_perm(B, H, H, 3, d, 160)))
    o = K.grouped_tile_order_i8(convs, 7).tolist()
    tiles = []
    for g, c in enumerate(convs):
        M = c["perm"].numel() if "perm" in c else B * H * H
        tiles += [(g << 24) | t for t in range(-(-M // 160) * (A // 128))]
    assert sorted(o) == sorted(tiles)
    taps = {g: K._tile_taps(B, H, H, c.get("k", 1), c.get("dil", 1), 160, c.get("perm"))
            for g, c in enumerate(convs)}
    cost = [int(taps[e >> 24][(e & 0xFFFFFF) // 2]) for e in o]
    assert cost == sorted(cost, reverse=True) and cost[0] == 9 and cost[-1] == 1
    # the permutation: the rate-18 branch's tiles average well under the raster tiles' taps
    raster = K._tile_taps(B, H, H, 3, 18, 160, None).float().mean()
    assert taps[3].float().mean() < 0.8 * raster
    assert torch.is_tensor(K.grouped_tile_order_i8(convs[:1], 2))


def test_grouped_tile_order_i8_branch_affine_cpu():
    """xcds = 8: the same tiles, each XCD (position % 8) dominated by one 3x3 branch (a
    branch's overflow past its XCD set's block count spills to the neighbours)."""
    from semantic_segmentation_server_amd.ops import hip_ops as K
    B, H = 2, 33
    convs = [dict(B=B, OH=H, OW=H, Cin=1024, Cout=256)]
    for d in (6, 12, 18):
        convs.append(dict(B=B, OH=H, OW=H, Cin=1024, Cout=256, k=3, dil=d,
                          perm=K.tap_group_perm(B, H, H, 3, d, 160)))
    a = K.grouped_tile_order_i8(convs, 7).tolist()
    b = K.grouped_tile_order_i8(convs, 7, xcds=8).tolist()
    assert sorted(a) == sorted(b)
    for x in range(8):
        gs = [e >> 24 for e in b[x::8] if e >> 24 > 0]
        assert max(gs.count(g) for g in set(gs)) >= 0.75 * len(gs)
