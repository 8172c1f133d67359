"""Whisper vocabulary: special-token ids, token text, tokenizer (oracle side).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restates whisper.cpp's `whisper_vocab` (special ids shifted for multilingual
models by `num_languages() - 98`), the marker strings it assigns to ids beyond
the file vocabulary ("[_EOT_]", "[_TT_n]", ...) that the reference glue strips
(src/transcribe.rs:205-240), and whisper.cpp's `tokenize()` (regex word split +
greedy longest-prefix match) used for `initial_prompt`
(src/transcribe.rs:384-386 -> params.set_initial_prompt).

Synthetic file vocabulary (no ggml files here): ids [0,26) are
'a'..'z', id 26 is ' ', ids [27, 27+26^3) are ' ' + 3 letters, the rest below
EOT are 4-letter words.  The same table is built in csrc/vocab.cpp.
"""
from __future__ import annotations

LANGS = ("en zh de es ru ko fr ja pt tr pl ca nl ar sv it id hi fi vi he uk el ms cs ro da hu ta no "
         "th ur hr bg lt la mi ml cy sk te fa lv bn sr az sl kn et mk br eu is hy ne mn bs kk sq sw "
         "gl mr pa si km sn yo so af oc ka be tg sd gu am yi lo uz fo ht ps tk nn mt sa lb my bo tl "
         "mg as tt haw ln ha ba jw su yue").split()
assert len(LANGS) == 100


def _letters(k: int, n: int) -> str:
    s = []
    for _ in range(n):
        s.append(chr(ord('a') + k % 26))
        k //= 26
    return "".join(reversed(s))


class Vocab:
    def __init__(self, n_vocab: int):
        self.n_vocab = n_vocab
        self.multilingual = n_vocab >= 51865
        self.num_languages = n_vocab - 51765 - (1 if self.multilingual else 0)
        eot, sot = 50256, 50257
        tr, tc, solm, prev, nosp, nt, beg = 50357, 50358, 50359, 50360, 50361, 50362, 50363
        if self.multilingual:
            eot += 1
            sot += 1
            dt = self.num_languages - 98
            tr, tc, solm, prev, nosp, nt, beg = (x + dt for x in (tr, tc, solm, prev, nosp, nt, beg))
        self.eot, self.sot, self.translate, self.transcribe = eot, sot, tr, tc
        self.solm, self.prev, self.nosp, self.not_, self.beg = solm, prev, nosp, nt, beg
        words = []
        for i in range(n_vocab):
            words.append(self._text(i))
        self.id_to_token = words
        self.token_to_id = {}
        for i, w in enumerate(words):
            self.token_to_id[w] = i             # whisper.cpp: token_to_id[word] = i (last wins)

    def _text(self, i: int) -> str:
        if i < self.eot:
            if i < 26:
                return chr(ord('a') + i)
            if i == 26:
                return " "
            if i < 27 + 26 ** 3:
                return " " + _letters(i - 27, 3)
            return _letters(i - 27 - 26 ** 3, 4)
        if i > self.beg:
            return "[_TT_%d]" % (i - self.beg)
        if i == self.eot:
            return "[_EOT_]"
        if i == self.sot:
            return "[_SOT_]"
        if i == self.translate:
            return "[_TRANSLATE_]"
        if i == self.transcribe:
            return "[_TRANSCRIBE_]"
        if i == self.solm:
            return "[_SOLM_]"
        if i == self.prev:
            return "[_PREV_]"
        if i == self.nosp:
            return "[_NOSP_]"
        if i == self.not_:
            return "[_NOT_]"
        if i == self.beg:
            return "[_BEG_]"
        if self.sot < i <= self.sot + self.num_languages:
            return "[_LANG_%s]" % LANGS[i - self.sot - 1]
        return "[_extra_token_%d]" % i

    def token_lang(self, lang_id: int) -> int:
        return self.sot + 1 + lang_id

    # whisper.cpp tokenize(): split with
    #   's|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+
    # then greedy longest-prefix match per word; unknown bytes are skipped.
    def split_words(self, text: str):
        out, i, n = [], 0, len(text)

        def isalpha(c):
            return c.isalpha()

        def isdigit(c):
            return c.isdigit()

        def isspace(c):
            return c.isspace()
        while i < n:
            m = None
            for suf in ("'s", "'t", "'re", "'ve", "'m", "'ll", "'d"):
                if text.startswith(suf, i):
                    m = suf
                    break
            if m is None:
                j = i + 1 if (text[i] == " " and i + 1 < n) else i
                for cls in (isalpha, isdigit, lambda c: not (isspace(c) or isalpha(c) or isdigit(c))):
                    if j < n and cls(text[j]):
                        k = j
                        while k < n and cls(text[k]):
                            k += 1
                        m = text[i:k]
                        break
                if m is None and isspace(text[i]):
                    k = i
                    while k < n and isspace(text[k]):
                        k += 1
                    # \s+(?!\S): a whitespace run not followed by non-space -> all but the last
                    # space when followed by a word, else the whole run.
                    if k < n and k - i > 1:
                        m = text[i:k - 1]
                    else:
                        m = text[i:k]
                if m is None:
                    m = text[i]
            out.append(m)
            i += len(m)
        return out

    def tokenize(self, text: str):
        toks = []
        for word in self.split_words(text):
            i, n = 0, len(word)
            while i < n:
                j = n
                found = False
                while j > i:
                    t = self.token_to_id.get(word[i:j])
                    if t is not None:
                        toks.append(t)
                        i = j
                        found = True
                        break
                    j -= 1
                if not found:
                    i += 1
        return toks
