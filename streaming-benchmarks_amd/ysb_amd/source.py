"""The events file as the reference's source reads it, handed to the GPU in place.

FileBasedDataSource mirrors `FileBasedDataSource.run` (flink-benchmarks/.../
AdvertisingTopologyNative.java:144-165: a BufferedReader over the events file, one record
per readLine) and the native runner's in-place mode (host/ysb_topology.cpp
`FileBasedDataSource::nextMapped`): the file is mapped read-only, the mapping registered with
the context once (ysb_host_register), and each batch -- the whole lines that fit in the
slot, cut where readLine cuts ("\\n", "\\r\\n", a lone "\\r") -- is submitted where it lies
(ysb_submit_raw_mapped: the copy kernel reads it over PCIe at any byte alignment and the GPU
splits its lines).  No byte of the file passes through a host copy.
"""
import mmap
import os

import numpy as np

PAGE = mmap.PAGESIZE


def complete_end(buf, start: int, have: int, at_eof: bool) -> int:
    """The end (relative to start) of the complete lines among buf[start:start + have]: up to
    the last terminator, everything at end of file; a '\\r' that ends the window may still be
    followed by '\\n', so it waits (FileBasedDataSource::completeEnd)."""
    if at_eof:
        return have
    q = have
    while q > 0:
        c = buf[start + q - 1]
        if c == 0x0A or (c == 0x0D and q < have):
            return q
        q -= 1
    raise ValueError("a line is longer than the batch buffer")


class FileBasedDataSource:
    """The events file, mapped read-only: `ranges(cap)` yields (offset, nbytes) of whole-line
    batches, back to back; `run(ctx, cap)` registers the mapping and submits every batch in
    place on alternating slots."""

    def __init__(self, path: str):
        self.path = path
        self.size = os.path.getsize(path)
        self._mm = None
        self.data = np.zeros(0, dtype=np.uint8)
        if self.size:
            with open(path, "rb") as f:
                self._mm = mmap.mmap(f.fileno(), 0, flags=mmap.MAP_SHARED, prot=mmap.PROT_READ)
            self.data = np.frombuffer(self._mm, dtype=np.uint8)
        self.bytes_read = 0
        self.batches = 0

    @property
    def mapping_bytes(self) -> int:
        """The registrable length: the mapping's whole pages (the copy reads whole 16-byte
        vectors, so the last batch may read past the file's end inside its last page)."""
        return (self.size + PAGE - 1) // PAGE * PAGE

    def ranges(self, cap: int):
        if cap <= 0:
            raise ValueError("cap must be positive")
        pos = 0
        while pos < self.size:
            have = min(cap, self.size - pos)
            end = complete_end(self.data, pos, have, pos + have >= self.size)
            yield pos, end
            pos += end

    def run(self, ctx, cap: int, rebase=None):
        """Every batch of the file through ctx (a YsbContext), in place; returns the bytes
        submitted.  At most two batches in flight (ysb_wait on the slot about to be reused)."""
        if not self.size:
            return 0
        ctx.host_register(self.data, self.mapping_bytes)
        try:
            slot = 0
            for off, nb in self.ranges(cap):
                ctx.submit_raw_mapped(self.data, off, nb, slot=slot)
                slot ^= 1
                ctx.wait(slot)
                self.bytes_read += nb
                self.batches += 1
            ctx.sync()
        finally:
            ctx.host_unregister(self.data)
        return self.bytes_read

    def close(self):
        self.data = np.zeros(0, dtype=np.uint8)
        if self._mm is not None:
            try:
                self._mm.close()
            except BufferError:   # a caller still holds a view of the mapping: it stays until freed
                pass
            self._mm = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
