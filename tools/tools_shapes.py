SHAPES = {
    "metric": ("crc32c", 65536, 65536, 0x4D43310000000005),
    "c2": ("crc32c", 65536, 4096, 0x4D43310000000002),
    "c3": ("crc64", 8192, 1 << 20, 0x4D43310000000003),
    "seg": ("crc64", 8192, 1 << 20, 0x4D43310000000003),
    "c4": ("crc32c", 262144, None, 0x4D43310000000004),
    "c5": ("crc32c", 1 << 20, 65536, 0x4D43310000000005),
    "msgs": ("crc32c", 262144, None, 0x4D43310000000004),   # C4's packets as Mercury messages, verified
    "xdr": ("crc32c", 262144, None, 0x4D43310000000004),    # C4's payloads as XDR iovec messages
}
