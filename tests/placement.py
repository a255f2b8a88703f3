"""Device placement helpers for the GPU tests (no GPU needed to import)."""


def bit31_offset(base: int, need: int) -> int:
    """Offset into an allocation starting at `base` (of at least 2 GiB + 2 *
    need bytes) of a 256-B aligned run of `need` bytes that lies entirely in
    the upper half [2^31, 2^32) of one 4 GiB block, so every address in it
    has bit 31 set: the allocation's own start if it qualifies, else the next
    such half (at most 2 GiB + need away).  Round 4's TN fault: the buffer
    descriptor's base went through readfirstlane's int and was sign-extended
    into the high word for exactly such addresses."""
    assert need + 256 <= 1 << 31
    need += 256   # room for the alignment step
    low = base & 0xFFFFFFFF   # offset inside the 4 GiB block
    if low >= 1 << 31 and low + need <= 1 << 32:
        off = 0
    elif low < 1 << 31:
        off = (1 << 31) - low
    else:
        off = (1 << 32) - low + (1 << 31)
    return off + (-(base + off)) % 256


def bit31_alloc_bytes(need: int) -> int:
    """Allocation size bit31_offset needs for a run of `need` bytes."""
    return (1 << 31) + 2 * (need + 256)
