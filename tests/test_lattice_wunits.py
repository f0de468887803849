"""The lattice step's w-unit partition (mfgp_lattice.inl: wst_first / wst_unit /
wst_pos / the unit cursor; mfgp_internal.h: lat_wsteps), restated on the host:
every 16-row step of F's lower triangle is streamed by exactly one unit, every
unit's share is within one step of the others', a block's partial slots never
collide, and the host's partial buffer (LAT_WU_MAX + nwb slots) holds them.
CPU only: the device's own result is checked by the -m gpu lattice tests
(test_gpu_lattice.py::test_lattice_split_and_w_units_vs_oracle)."""
import pytest

LAT_WU_MAX = 512
LAT_NWB_MAX = 256


def lat_wsteps(n0):
    C, nwb = (n0 + 15) // 16, (n0 + 63) // 64
    return nwb * C - 2 * nwb * (nwb - 1)


def plan(n0, U):
    """Per unit: the blocks it streams (in order) and its step count; per block the
    unit range and slots of its partials -- the device's arithmetic step by step."""
    C, nwb = (n0 + 15) // 16, (n0 + 63) // 64
    K2 = 2 * C - 4 * (nwb - 1)
    S = (nwb // 2) * K2 + (nwb & 1) * (C - 4 * (nwb // 2))

    def first(jb):
        return jb * K2 if 2 * jb < nwb else (nwb - 1 - jb) * K2 + C - 4 * (nwb - 1 - jb)

    def unit(s):
        return ((s + 1) * U - 1) // S

    def pos(jb):
        return 2 * jb if 2 * jb < nwb else 2 * (nwb - 1 - jb) + 1

    cover = [0] * nwb
    slots = {}
    lens = []
    for u in range(U):
        s0, s1 = u * S // U, (u + 1) * S // U
        T = s1 - s0
        lens.append(T)
        p = s0 // K2
        rem = s0 - p * K2
        odd = rem >= C - 4 * p
        jb = nwb - 1 - p if odd else p
        st = rem - (C - 4 * p) if odd else rem
        nb = C - 4 * jb
        # the wait for the compact rows covers every row the unit streams
        lo = 64 * jb + 16 * st
        lo_wait = min(lo, 64 * (p + 1)) if st + T > C - 4 * jb else lo
        segs = []
        for t in range(T):
            cover[jb] += 1
            assert 64 * jb + 16 * st >= lo_wait
            if st + 1 == nb or t + 1 == T:
                segs.append(jb)
            if t + 1 < T:
                st += 1
                if st == nb:
                    st = 0
                    if odd:
                        p += 1
                        jb = p
                    else:
                        jb = nwb - 1 - p
                    odd = not odd
                    nb = C - 4 * jb
        assert len(segs) <= LAT_NWB_MAX
        for b in segs:
            f = first(b)
            ua, ub = unit(f), unit(f + C - 4 * b - 1)
            assert ua <= u <= ub
            sl = u + pos(b)
            assert sl not in slots, (n0, U, u, b, slots[sl])
            slots[sl] = (u, b)
    return S, cover, slots, lens, C, nwb


@pytest.mark.parametrize("n0", [1, 15, 16, 17, 63, 64, 65, 127, 300, 1000, 2040, 2047, 4096, 8184])
@pytest.mark.parametrize("U", [1, 2, 3, 7, 32, 64, 256, 512])
def test_w_unit_partition(n0, U):
    U = max(1, min(U, LAT_WU_MAX, lat_wsteps(n0)))   # the host's clamp
    S, cover, slots, lens, C, nwb = plan(n0, U)
    assert S == lat_wsteps(n0)
    assert cover == [C - 4 * jb for jb in range(nwb)]     # every step exactly once
    assert max(lens) - min(lens) <= 1                      # equal shares
    assert max(slots) < LAT_WU_MAX + nwb                   # fits the host's partial buffer


def test_host_unit_counts_share_the_launch():
    """The host's rule (mfgp_capi.hip): two units per CU over the launch, each GP's
    count by its F steps, clamped to [1, min(LAT_WU_MAX, steps)]."""
    def counts(n0s, total=512):
        st = [lat_wsteps(n) for n in n0s]
        tot = sum(st)
        return [max(1, min((total * s + tot // 2) // tot, LAT_WU_MAX, s)) for s in st]
    assert counts([2040] * 8) == [64] * 8
    assert counts([2040]) == [512]
    assert sum(counts([2040] * 32)) == 512
    assert counts([10, 2040]) == [1, 512]
