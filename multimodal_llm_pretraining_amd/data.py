"""Synthetic datasets of the benchmark (§8(a) row a15), restating
src/benchmarking/data.py:8-21 (text) and :45-77 (multimodal).

Differences, both deliberate and documented in DESIGN.md:
* samples are generated lazily and deterministically per index from (seed, index)
  instead of materialising all of them up front (the reference's 20,000 fp32 images
  at 224² are 12 GB of host RAM); distributions are the reference's: ids ~ U{0..V-1},
  pixels ~ U[0,1), attention_mask = 1, labels = ids;
* the multimodal set pre-expands the image placeholder to `image_tokens` slots (196
  for ViT-B/16 at 224²) with label -100 on those slots — the transformers-4.47 LLaVA
  expansion the build restates; text ids then avoid the image token.
  With image_tokens=1 the reference layout (one <image> token, labels = ids) is kept.
"""

from __future__ import annotations

import torch
from torch.utils.data import Dataset


def _gen(seed: int, index: int) -> torch.Generator:
    return torch.Generator().manual_seed((seed * 1_000_003 + index) & 0x7FFF_FFFF_FFFF_FFFF)


class DummyTextModelingDataset(Dataset):
    def __init__(self, vocab_size: int, sequence_length: int, num_samples: int = 50_000,
                 seed: int = 0) -> None:
        super().__init__()
        self.vocab_size, self.sequence_length = vocab_size, sequence_length
        self.num_samples, self.seed = num_samples, seed

    def __len__(self):
        return self.num_samples

    def __getitem__(self, index):
        if not 0 <= index < self.num_samples:
            raise IndexError(index)
        ids = torch.randint(0, self.vocab_size, (self.sequence_length,), generator=_gen(self.seed, index))
        return {"input_ids": ids, "labels": ids.clone()}


class DummyMultimodalLanguageModelingDataset(Dataset):
    def __init__(self, vocab_size: int, sequence_length: int, image_size: int,
                 num_samples: int = 20_000, image_token_id: int = 32000, image_tokens: int = 1,
                 seed: int = 0) -> None:
        super().__init__()
        if not 1 <= image_tokens < sequence_length:
            raise ValueError("need 1 <= image_tokens < sequence_length")
        self.vocab_size, self.sequence_length, self.image_size = vocab_size, sequence_length, image_size
        self.num_samples, self.image_token_id, self.image_tokens = num_samples, image_token_id, image_tokens
        self.seed = seed

    def __len__(self):
        return self.num_samples

    def __getitem__(self, index):
        if not 0 <= index < self.num_samples:
            raise IndexError(index)
        g = _gen(self.seed, index)
        n_text = self.sequence_length - self.image_tokens
        if self.image_tokens == 1:  # reference layout
            text = torch.randint(0, self.vocab_size, (n_text,), generator=g)
        else:  # U{0..V-1} \ {image_token_id}
            text = torch.randint(0, self.vocab_size - 1, (n_text,), generator=g)
            text = text + (text >= self.image_token_id).long()
        ids = torch.cat([torch.full((self.image_tokens,), self.image_token_id), text])
        labels = ids.clone()
        if self.image_tokens > 1:
            labels[: self.image_tokens] = -100
        pixels = torch.rand((3, self.image_size, self.image_size), generator=g)
        return {"attention_mask": torch.ones_like(ids), "pixel_values": pixels,
                "input_ids": ids, "labels": labels}


class PrefetchLoader:
    """The data-loader side of the step (what `trainer.get_train_dataloader()` feeds
    `benchmark_acc_optim_times`, src/benchmarking/step_time.py:49-56): micro-batches of
    `batch_size` samples of `dataset`, indices strided over the data-parallel ranks
    (DistributedSampler order without shuffling), collated and pinned by a background
    thread `depth` batches ahead — torch's CPU ops release the GIL, so generating the next
    batch overlaps the step like DataLoader workers do.  Iterates forever (wrapping the
    index range): the benchmark asks for as many batches as it times."""

    def __init__(self, dataset, batch_size: int, rank: int = 0, world: int = 1, depth: int = 2,
                 pin: bool = True):
        import queue
        import threading

        self.ds, self.bs, self.rank, self.world, self.pin = dataset, batch_size, rank, world, pin
        self.q: queue.Queue = queue.Queue(maxsize=max(1, depth))
        self._stop = threading.Event()
        self._next = 0
        self.thread = threading.Thread(target=self._run, name="mmpt-loader", daemon=True)
        self.thread.start()

    def _batch(self) -> dict:
        n = len(self.ds)
        idx = [((self._next + i) * self.world + self.rank) % n for i in range(self.bs)]
        self._next += self.bs
        samples = [self.ds[i] for i in idx]
        out = {}
        for k in samples[0]:
            t = torch.stack([s[k] for s in samples])
            out[k] = t.pin_memory() if self.pin and torch.cuda.is_available() else t
        return out

    def _run(self) -> None:
        try:
            while not self._stop.is_set():
                b = self._batch()
                while not self._stop.is_set():
                    try:
                        self.q.put(b, timeout=0.1)
                        break
                    except Exception:  # queue.Full
                        continue
        except BaseException as e:  # surfaced by __next__
            self.q.put(e)

    def __iter__(self):
        return self

    def __next__(self) -> dict:
        b = self.q.get()
        if isinstance(b, BaseException):
            raise RuntimeError("data loader thread failed") from b
        return b

    def close(self) -> None:
        self._stop.set()
        self.thread.join(timeout=5)
