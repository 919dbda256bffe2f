"""Experiment (not product): the batch pass's per-compression time.

Times sha256_lists_kernel (mirsha_digest_lists_device) over device-resident
request digests for list counts from one wave to 2x config 2's 52,429 and
list lengths 4 / 20 / 40 digests (3 / 11 / 21 compressions per chain), with
the engine's HIP events on its stream.  The slope over list length at a fixed
count is the per-compression time of the chain; one wave alone gives its
latency floor, config 2's count shows what the placement adds.

    python tools/exp_lists.py > gpurun_out/lists.jsonl
"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mirbft_amd import Engine  # noqa: E402
from mirbft_amd.engine import KERNEL_LISTS  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n_dig = 1 << 20
    d_dig = torch.randint(0, 256, (n_dig * 32,), dtype=torch.uint8, device=dev)
    for bs in (4, 20, 40):
        for n_lists in (64, 1024, 16384, 52429, 104858):
            entries = n_lists * bs
            idx = (torch.arange(entries, dtype=torch.int64, device=dev) * 7919 % n_dig).to(torch.int32)
            first = torch.arange(0, entries + 1, bs, dtype=torch.int32, device=dev)
            out = torch.empty(n_lists * 32, dtype=torch.uint8, device=dev)

            def run():
                eng.digest_lists_device(d_dig.data_ptr(), n_dig, idx.data_ptr(), first.data_ptr(), n_lists, entries,
                                        out.data_ptr())

            for _ in range(10):
                run()
            torch.cuda.synchronize(dev)
            eng.set_timing(True)
            eng.set_timing_mask([KERNEL_LISTS])
            eng.reset_timing()
            for _ in range(50):
                run()
            torch.cuda.synchronize(dev)
            n, ms = eng.kernel_time(KERNEL_LISTS)
            eng.set_timing(False)
            blocks = (32 * bs + 72) // 64
            us = ms / n * 1e3
            print(json.dumps({"list_digests": bs, "compressions_per_chain": blocks, "lists": n_lists,
                              "waves": -(-n_lists // 64), "kernel_us": round(us, 2),
                              "us_per_compression": round(us / blocks, 3)}), flush=True)


if __name__ == "__main__":
    main()
