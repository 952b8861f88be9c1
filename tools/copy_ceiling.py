"""The device-copy ceiling the copy-out is judged against.

tm_copy_out moves C3's match ids from the stage rows to the CSR output: 8M
topics x 56.0 ids x 4 B read + the same written = 3.58 GB per launch.  This
times a plain device-to-device copy of the same byte count (torch's copy_,
i.e. the runtime's blit kernel), so the copy-out's rate
can be read as a fraction of what a pure stream copy reaches on this HBM.
Prints one JSON line.
"""
import json
import sys

import torch


def main():
    ids = int(sys.argv[1]) if len(sys.argv) > 1 else 8_000_000 * 56
    dev = torch.device("cuda", 0)
    src = torch.randint(0, 1 << 30, (ids,), dtype=torch.int32, device=dev)
    dst = torch.empty_like(src)
    out = {"ids": ids, "bytes_read_plus_written": 8 * ids}
    for name, fn in (("copy_", lambda: dst.copy_(src)),):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ms = []
        for _ in range(20):
            a.record()
            fn()
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b))
        ms.sort()
        med = ms[len(ms) // 2]
        out[name] = {"ms_median": med, "ms_min": ms[0], "TB_s": 8 * ids / med / 1e9}
    assert torch.equal(dst, src)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
