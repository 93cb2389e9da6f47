"""Host restatements of two device data layouts (no GPU): the LDS images of k_wgrad_dma
(anr_tgemm.hip: 32-sample x 256-column bf16 images, 16-B chunks XOR-swizzled per row, filled by
LDS-DMA and read by ds_read_b64_tr_b16) and the chain kernels' output-neuron order (anr_tchain.hip
tc_nrn). Each check restates the kernel's index arithmetic and asserts the property the kernel relies
on: every element written exactly once and read back from where it was written, conflict-free LDS
banking (MI355X_MICROARCH.md §LDS: ds_read_b64 serves two 32-lane halves, bank = (address / 4) mod 64),
and 8 consecutive neurons per lane for the 16-B row stores."""
import numpy as np


def wd_swz(r):
    return 2 * ((r & 3) | (((r >> 3) & 1) << 2))


def test_wgrad_dma_image_fill_is_a_bijection():
    # a stage image: 16 pieces of 1 KiB (8 waves x 2), lane L of piece p writes LDS bytes p*1024 + 16 L
    seen = np.zeros((32, 32), int)  # (row, logical chunk)
    for piece in range(16):
        for lane in range(64):
            off = piece * 1024 + 16 * lane
            r, cp = off // 512, (off % 512) // 16
            assert r == 2 * piece + (lane >> 5) and cp == (lane & 31)
            c = cp ^ wd_swz(r)  # the logical chunk the lane fetches from global memory
            assert 0 <= c < 32
            seen[r, c] += 1
    assert np.all(seen == 1)


def _frag_addresses(c0):
    """Byte addresses of wd_frag's two ds_read_b64_tr_b16 per lane, and the (row, column) each reads."""
    out = []
    for lane in range(64):
        g, q, p = lane >> 4, (lane >> 2) & 3, lane & 3
        c = c0 + 4 * p
        reads = []
        for r in (8 * g + q, 8 * g + q + 4):
            a = r * 512 + (((c >> 3) ^ wd_swz(r)) << 4) + (c & 7) * 2
            reads.append((a, r, c))
        out.append(reads)
    return out


def test_wgrad_dma_fragment_reads_hit_the_written_elements():
    for c0 in range(0, 256, 16):
        for lane, reads in enumerate(_frag_addresses(c0)):
            for a, r, c in reads:
                # the 8 B at a hold columns c .. c + 3 of row r: undo the swizzle of the fill
                row, cp, within = a // 512, (a % 512) // 16, (a % 16) // 2
                assert row == r and (cp ^ wd_swz(row)) * 8 + within == c and within in (0, 4)


def test_wgrad_dma_fragment_reads_are_bank_conflict_free():
    for c0 in range(0, 256, 16):
        addrs = _frag_addresses(c0)
        for k in range(2):  # each of the two tr reads
            for half in range(2):
                banks = []
                for lane in range(32 * half, 32 * half + 32):
                    a = addrs[lane][k][0]
                    banks += [(a // 4) % 64, (a // 4 + 1) % 64]  # 8 B = 2 banks
                assert len(set(banks)) == 64, (c0, k, half)


def tc_nrn(o, m):
    return 32 * (o >> 1) + 8 * (m >> 2) + 4 * (o & 1) + (m & 3)


def test_chain_output_order():
    # every output neuron of a 16-block layer exactly once
    got = sorted(tc_nrn(o, m) for o in range(16) for m in range(16))
    assert got == list(range(256))
    # lane h of the C fragments of out-blocks 2s, 2s + 1 holds (rows 4h + r) the 8 consecutive neurons
    # 32 s + 8 h + 0..7: one 16-B store, and the natural-order B fragment of the next layer's k-step s
    for s in range(8):
        for h in range(4):
            run = [tc_nrn(2 * s, 4 * h + r) for r in range(4)] + [tc_nrn(2 * s + 1, 4 * h + r) for r in range(4)]
            assert run == list(range(32 * s + 8 * h, 32 * s + 8 * h + 8))
    # feature || alpha: block 16 row 0 is neuron 256 (alpha_fc), read by lane h == 0, element 0
    assert tc_nrn(16, 0) == 256


def test_chain_mask_bit_tree():
    # 16 words with bits 0 / 16 set as a lane's (half != 0) flags -> 32 bits: word k at k and 16 + k
    rng = np.random.default_rng(3)
    for _ in range(50):
        t = [int(x) for x in (rng.integers(0, 2, 16) | (rng.integers(0, 2, 16) << 16))]
        a = [t[k] | (t[k + 8] << 8) for k in range(8)]
        b = [a[k] | (a[k + 4] << 4) for k in range(4)]
        c0, c1 = b[0] | (b[2] << 2), b[1] | (b[3] << 2)
        f = (c0 | (c1 << 1)) & 0xffffffff
        for k in range(16):
            assert (f >> k) & 1 == t[k] & 1 and (f >> (16 + k)) & 1 == (t[k] >> 16) & 1
