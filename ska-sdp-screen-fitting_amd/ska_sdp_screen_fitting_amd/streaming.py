"""Device -> FITS streaming for Screen.write.

The kernels store big-endian float32 (SF_EVAL_BIG_ENDIAN), i.e. the FITS
byte order, so the host never converts: each batch of time rows is evaluated
into a device buffer, copied asynchronously into one of two pinned host
buffers on a copy stream, and written to the file by a writer thread while
the GPU evaluates the next batch.
"""

import queue
import threading


class PinnedPipeline:
    """Overlap: evaluate batch k+1 | copy batch k | write batch k-1."""

    def __init__(self, torch, device, max_batch_bytes):
        self.torch = torch
        self.dev = device
        self.cap = int(max_batch_bytes)
        self.host = [torch.empty(self.cap, dtype=torch.uint8, pin_memory=True)
                     for _ in range(2)]
        self.devbuf = [torch.empty(self.cap, dtype=torch.uint8, device=device)
                       for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(device)
        self.copied = [None, None]
        self.free = [threading.Event(), threading.Event()]
        for e in self.free:
            e.set()
        self.q = queue.Queue()
        self.err = None
        self.thread = threading.Thread(target=self._writer, daemon=True)
        self.thread.start()
        self.k = 0

    def _writer(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            slot, nbytes, writer = item
            try:
                self.copied[slot].synchronize()
                writer.write_raw(memoryview(self.host[slot].numpy())[:nbytes])
            except Exception as exc:  # surfaced in close()
                self.err = exc
            finally:
                self.free[slot].set()

    def device_buffer(self, nbytes):
        """Next device buffer (uint8 view of >= nbytes)."""
        slot = self.k % 2
        assert nbytes <= self.cap
        return slot, self.devbuf[slot][:nbytes]

    def submit(self, slot, nbytes, writer):
        """After the kernel writing devbuf[slot] was enqueued on the current
        stream: copy it to pinned memory and hand it to the writer thread."""
        torch = self.torch
        self.free[slot].wait()      # the writer is done with host[slot]
        self.free[slot].clear()
        cur = torch.cuda.current_stream(self.dev)
        self.copy_stream.wait_stream(cur)
        with torch.cuda.stream(self.copy_stream):
            self.host[slot][:nbytes].copy_(self.devbuf[slot][:nbytes], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        # the next kernel into devbuf[slot] must wait for this copy
        cur.wait_event(ev)
        self.copied[slot] = ev
        self.q.put((slot, nbytes, writer))
        self.k += 1

    def close(self):
        self.q.put(None)
        self.thread.join()
        if self.err is not None:
            raise self.err
