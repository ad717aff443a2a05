"""Batch assembly of the data path (reference: matcha/data_management/ljspeech_datamodule.py:84-109,
LJSpeechDataModule.collate), plus the length bucketing the reference lacks (BASELINE
config 5 "bucketed padding").

`collate(batch)` returns exactly the reference's dict (x zero-padded [B, Tx_max] int64, y zero-padded
[B, n_mels, Ty_max], x_lengths / y_lengths [B]).  `LengthBucketBatchSampler` groups utterances of
similar mel length so the decoder runs at a smaller padded T; for data parallelism it sorts each
GLOBAL batch (batch_size x world) by length and deals it round-robin, so every rank gets one
utterance of every length stratum (balanced padded T, identical batch counts on every rank).
Bucketing changes what the decoder sees (GroupNorm statistics run over the padded T, decoder.py:58-66),
so the reference's unbucketed order stays available: `shuffle=True, bucket_batches=0`.
The file-reading Dataset (text cleaners + wav IO) is not on the hot path; MelSpectrogram
(matcha/utils/audio_process.py) computes the features on the GPU in batch.
"""
from __future__ import annotations

import torch
from torch.nn.utils.rnn import pad_sequence


def _round_up(n: int, q: int) -> int:
    return -(-n // q) * q


def collate(batch, x_quantum: int = 1, y_quantum: int = 1, n_vocab: int | None = None):
    """ljspeech_datamodule.py:84-109: items {"x": int64 [Tx_i], "y": [n_mels, Ty_i], "x_lengths",
    "y_lengths"} -> padded batch dict (padding value 0).

    x_quantum / y_quantum > 1 pad Tx_max / Ty_max further, up to a multiple of the quantum, so that
    batches fall into a few padded shapes and the graph-mode Trainer replays a cached step graph
    instead of capturing one per batch (its LRU cache, TrainConfig.graph_cache).  1 (default) is the
    reference's padding to the batch maximum; a larger padded T only adds masked frames, but the
    decoder's GroupNorm statistics run over the padded length (decoder.py:58-66), as with bucketing.

    n_vocab: when given, token ids outside [0, n_vocab) raise ValueError here, on the host (the
    reference's nn.Embedding would hit a device assert; the HIP embedding poisons such rows with NaN)."""
    x = [item["x"] for item in batch]
    if n_vocab is not None:
        for i, xi in enumerate(x):
            if xi.numel() and (int(xi.min()) < 0 or int(xi.max()) >= n_vocab):
                raise ValueError(f"collate: item {i} has token ids outside [0, {n_vocab})")
    x_lengths = torch.tensor([int(item["x_lengths"]) for item in batch])
    y_lengths = torch.tensor([int(item["y_lengths"]) for item in batch])
    x_padded = pad_sequence(x, batch_first=True, padding_value=0)
    # time-major views for pad_sequence, back to [B, n_mels, T] (the reference's transposes, :104-105)
    y_padded = pad_sequence([item["y"].transpose(0, 1) for item in batch], batch_first=True,
                            padding_value=0).transpose(1, 2)
    tx, ty = _round_up(x_padded.shape[1], x_quantum), _round_up(y_padded.shape[2], y_quantum)
    if tx != x_padded.shape[1]:
        x_padded = torch.nn.functional.pad(x_padded, (0, tx - x_padded.shape[1]))
    if ty != y_padded.shape[2]:
        y_padded = torch.nn.functional.pad(y_padded, (0, ty - y_padded.shape[2]))
    return {"x": x_padded, "x_lengths": x_lengths, "y": y_padded, "y_lengths": y_lengths}


class LengthBucketBatchSampler(torch.utils.data.Sampler):
    """Yields this rank's index lists.  Per epoch (seed + epoch): shuffle all indices, cut them into
    pools of `bucket_batches` global batches, sort each pool by length (descending), cut it into
    global batches of batch_size * num_replicas, shuffle the global batches, and give rank r the
    entries r, r + num_replicas, ... of each (length-sorted) global batch.  drop_last semantics: the
    tail that does not fill a global batch is dropped, so every rank yields len(self) batches.
    bucket_batches=0 disables the sorting (plain shuffled batches, the reference's order)."""

    def __init__(self, lengths, batch_size: int, num_replicas: int = 1, rank: int = 0, bucket_batches: int = 32,
                 shuffle: bool = True, seed: int = 0):
        if batch_size < 1 or num_replicas < 1 or not 0 <= rank < num_replicas:
            raise ValueError("LengthBucketBatchSampler: bad batch_size / num_replicas / rank")
        self.lengths = torch.as_tensor(lengths, dtype=torch.int64)
        self.batch_size = batch_size
        self.num_replicas = num_replicas
        self.rank = rank
        self.bucket_batches = bucket_batches
        self.shuffle = shuffle
        self.seed = seed
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __len__(self) -> int:
        return len(self.lengths) // (self.batch_size * self.num_replicas)

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        n = len(self.lengths)
        order = torch.randperm(n, generator=g) if self.shuffle else torch.arange(n)
        gb = self.batch_size * self.num_replicas
        order = order[: len(self) * gb]
        globals_ = []
        if self.bucket_batches > 0:
            pool = gb * self.bucket_batches
            for s in range(0, len(order), pool):
                chunk = order[s: s + pool]
                # stable sort on (-length) so equal lengths keep the shuffled order
                chunk = chunk[torch.sort(-self.lengths[chunk], stable=True).indices]
                globals_ += list(chunk.split(gb))
            if self.shuffle:
                globals_ = [globals_[i] for i in torch.randperm(len(globals_), generator=g).tolist()]
        else:
            globals_ = list(order.split(gb))
        for gbatch in globals_:
            yield gbatch[self.rank:: self.num_replicas].tolist()
