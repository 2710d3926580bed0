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
