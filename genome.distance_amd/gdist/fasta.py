"""FASTA records as FastaInputStream yields them (org.theseed.sequence.Sequence).

A record is `>label comment` followed by sequence lines; the label is the
text up to the first whitespace, the comment the rest of the header line.
"""
from __future__ import annotations

import dataclasses
from typing import Iterable, Iterator, TextIO


@dataclasses.dataclass
class Sequence:
    label: str
    comment: str
    sequence: str

    def getLabel(self) -> str:
        return self.label

    def getComment(self) -> str:
        return self.comment

    def getSequence(self) -> str:
        return self.sequence


def read_fasta(stream: TextIO | Iterable[str]) -> Iterator[Sequence]:
    label = comment = None
    parts: list[str] = []
    for line in stream:
        line = line.rstrip("\r\n")
        if line.startswith(">"):
            if label is not None:
                yield Sequence(label, comment, "".join(parts))
            head = line[1:]
            bits = head.split(None, 1)
            label = bits[0] if bits else ""
            comment = bits[1].strip() if len(bits) > 1 else ""
            parts = []
        elif label is not None:
            parts.append(line.strip())
    if label is not None:
        yield Sequence(label, comment, "".join(parts))


def write_fasta(records: Iterable[Sequence], out: TextIO, width: int = 60) -> None:
    for r in records:
        out.write(f">{r.label} {r.comment}\n" if r.comment else f">{r.label}\n")
        for i in range(0, len(r.sequence), width):
            out.write(r.sequence[i:i + width] + "\n")
