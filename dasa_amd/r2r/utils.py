"""The parts of r2r_src/utils.py the policy path uses (angle features, masks) and the word Tokenizer
the speaker decodes with (utils.py:129-227); the BERT tokenizer and dataset IO stay with the reference
(feature readers: dasa_amd/features.py, navigation graphs: dasa_amd/r2r/eval.py)."""
import math
import re
import string
import sys
from collections import defaultdict

import numpy as np
import torch

from .param import args

padding_idx = 0   # base_vocab.index('<PAD>') (utils.py:22-24); BERT [PAD] is 0 too


def angle_feature(heading, elevation):
    """utils.py:361-368."""
    return np.array([math.sin(heading), math.cos(heading), math.sin(elevation), math.cos(elevation)]
                    * (args.angle_feat_size // 4), dtype=np.float32)


def length2mask(length, size=None, device=None):
    """utils.py:503-508: True where index > len-1, on the compute device."""
    size = int(max(length)) if size is None else size
    lens = torch.as_tensor(list(length), dtype=torch.int64)
    mask = torch.arange(size, dtype=torch.int64).unsqueeze(0) > (lens - 1).unsqueeze(1)
    # pinned + non_blocking: the copy is queued on the stream instead of syncing the host with it
    return mask.pin_memory().to(device if device is not None else torch.device("cuda"), non_blocking=True)


def read_vocab(path):
    """utils.py:253-256."""
    with open(path) as f:
        return [word.strip() for word in f.readlines()]


class Tokenizer(object):
    """utils.py:129-227: word vocabulary (train_vocab.txt) plus <BOS>; unknown words map to <UNK>."""
    SENTENCE_SPLIT_REGEX = re.compile(r"(\W+)")

    def __init__(self, vocab=None, encoding_length=20):
        self.encoding_length = encoding_length
        self.vocab = vocab
        self.word_to_index = {}
        self.index_to_word = {}
        if vocab:
            for i, word in enumerate(vocab):
                self.word_to_index[word] = i
            new_w2i = defaultdict(lambda: self.word_to_index["<UNK>"])
            new_w2i.update(self.word_to_index)
            self.word_to_index = new_w2i
            for key, value in self.word_to_index.items():
                self.index_to_word[value] = key
        self.add_word("<BOS>")

    def finalize(self):
        self.word_to_index = dict(self.word_to_index)

    def add_word(self, word):
        assert word not in self.word_to_index
        self.word_to_index[word] = self.vocab_size()
        self.index_to_word[self.vocab_size()] = word

    @staticmethod
    def split_sentence(sentence):
        toks = []
        for word in [s.strip().lower() for s in Tokenizer.SENTENCE_SPLIT_REGEX.split(sentence.strip())
                     if len(s.strip()) > 0]:
            if all(c in string.punctuation for c in word) and not all(c in "." for c in word):
                toks += list(word)
            else:
                toks.append(word)
        return toks

    def vocab_size(self):
        return len(self.index_to_word)

    def encode_sentence(self, sentence, max_length=None):
        if max_length is None:
            max_length = self.encoding_length
        if len(self.word_to_index) == 0:
            sys.exit("Tokenizer has no vocab")
        encoding = [self.word_to_index["<BOS>"]]
        for word in self.split_sentence(sentence):
            encoding.append(self.word_to_index[word])
        encoding.append(self.word_to_index["<EOS>"])
        if len(encoding) <= 2:
            return None
        if len(encoding) < max_length:
            encoding += [self.word_to_index["<PAD>"]] * (max_length - len(encoding))
        elif len(encoding) > max_length:
            encoding[max_length - 1] = self.word_to_index["<EOS>"]
        return np.array(encoding[:max_length])

    def decode_sentence(self, encoding, length=None):
        sentence = []
        if length is not None:
            encoding = encoding[:length]
        for ix in encoding:
            if ix == self.word_to_index["<PAD>"]:
                break
            sentence.append(self.index_to_word[ix])
        return " ".join(sentence)

    def shrink(self, inst):
        if len(inst) == 0:
            return inst
        end = np.argmax(np.array(inst) == self.word_to_index["<EOS>"])
        start = 1 if len(inst) > 1 and inst[0] == self.word_to_index["<BOS>"] else 0
        return inst[start: end]
