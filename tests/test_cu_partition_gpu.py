"""CU shares of ranks that share one device (kctc_set_cu_partition,
DESIGN.md §6): each share is a contiguous range of CU-mask bits, and a mask
bit names one physical CU, so the shares must be disjoint CU sets that
together stay within the device, each spread over every XCD (bit b: XCD b mod
8).  Probed with blocks on streams built from the same masks
(kctc_cu_partition_probe), each reporting its XCC_ID and HW_ID."""
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(120)]


@pytest.mark.parametrize("nparts", [2, 4])
def test_partitions_are_disjoint(kctc, gpu, nparts):
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    sets = [set(int(v) for v in kctc.cu_partition_probe(p, nparts)) for p in range(nparts)]
    for p, s in enumerate(sets):
        assert 0 < len(s) <= cus // nparts, (p, len(s))
        assert len({v >> 16 for v in s}) == 8, f"share {p} does not reach every XCD"
    for i in range(nparts):
        for j in range(i + 1, nparts):
            assert not (sets[i] & sets[j]), f"shares {i} and {j} overlap: {sorted(sets[i] & sets[j])[:8]}"
