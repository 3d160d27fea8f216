"""English text -> espeak-ng style IPA (en-us) for piper voices with phoneme_type "espeak".

go-piper phonemises through espeak-ng (reference backend/go/tts/piper.go:20-49; the espeak-ng data
path is set in pkg/model/initializers.go:434-437).  espeak-ng is not in this image, so this module
is a rule-based stand-in that writes what espeak-ng's en-us voice writes for common English: the
same phoneme inventory (IPA code points, length mark "ː", stress marks "ˈ" / "ˌ" placed before the
stressed vowel, "ɚ" / "ɜː" r-colouring, the en-us flap "ɾ"), words separated by " ", punctuation
kept as its own phoneme.  A lexicon covers the function words and frequent irregular words (their
espeak-ng spellings); everything else goes through letter-to-sound rules, a stress heuristic and
unstressed-vowel reduction.  Output outside a voice's phoneme_id_map is folded onto phonemes it
has (fold()).  Parity with real espeak-ng is unpinned (no espeak-ng here); tests/test_piper.py
checks the inventory and the dictionary readings of common words.
"""
from __future__ import annotations

import re
from typing import Dict, List

# ---------------------------------------------------------------- lexicon (espeak-ng en-us forms)
LEXICON: Dict[str, str] = {
    "a": "ɐ", "an": "ɐn", "the": "ðə", "and": "ænd", "of": "ʌv", "to": "tə", "in": "ɪn", "is": "ɪz",
    "it": "ɪt", "you": "juː", "that": "ðæt", "he": "hiː", "was": "wʌz", "for": "fɔːɹ", "on": "ɑːn",
    "are": "ɑːɹ", "as": "æz", "with": "wɪð", "his": "hɪz", "they": "ðeɪ", "i": "aɪ", "at": "æt",
    "be": "biː", "this": "ðɪs", "have": "hæv", "from": "fɹʌm", "or": "ɔːɹ", "one": "wˈʌn", "had": "hæd",
    "by": "baɪ", "word": "wˈɜːd", "but": "bˌʌt", "not": "nˌɑːt", "what": "wˌʌt", "all": "ˈɔːl",
    "were": "wɜː", "we": "wiː", "when": "wˌɛn", "your": "jʊɹ", "can": "kæn", "said": "sˈɛd",
    "there": "ðɛɹ", "use": "jˈuːz", "each": "ˈiːtʃ", "which": "wˌɪtʃ", "she": "ʃiː", "do": "dˈuː",
    "does": "dˈʌz", "how": "hˌaʊ", "their": "ðɛɹ", "if": "ɪf", "will": "wɪl", "up": "ˌʌp",
    "other": "ˈʌðɚ", "about": "ɐbˈaʊt", "out": "ˈaʊt", "many": "mˈɛni", "then": "ðˈɛn", "them": "ðˌɛm",
    "these": "ðiːz", "so": "sˌoʊ", "some": "sˌʌm", "her": "hɜː", "would": "wʊd", "make": "mˈeɪk",
    "like": "lˈaɪk", "him": "hˌɪm", "into": "ˌɪntʊ", "time": "tˈaɪm", "has": "hɐz", "look": "lˈʊk",
    "two": "tˈuː", "more": "mˈoːɹ", "go": "ɡˌoʊ", "see": "sˈiː", "no": "nˈoʊ", "way": "wˈeɪ",
    "could": "kʊd", "people": "pˈiːpəl", "my": "maɪ", "than": "ðɐn", "first": "fˈɜːst",
    "water": "wˈɔːɾɚ", "been": "bˌɪn", "who": "hˌuː", "now": "nˈaʊ", "its": "ɪts", "day": "dˈeɪ",
    "did": "dˈɪd", "get": "ɡɛt", "come": "kˈʌm", "made": "mˈeɪd", "may": "mˈeɪ", "part": "pˈɑːɹt",
    "yes": "jˈɛs", "good": "ɡˈʊd", "hello": "həlˈoʊ", "world": "wˈɜːld", "test": "tˈɛst",
    "voice": "vˈɔɪs", "speech": "spˈiːtʃ", "please": "plˈiːz", "thank": "θˈæŋk", "thanks": "θˈæŋks",
    "computer": "kəmpjˈuːɾɚ", "give": "ɡˈɪv", "live": "lˈɪv", "love": "lˈʌv", "done": "dˈʌn",
    "gone": "ɡˈɔːn", "only": "ˈoʊnli", "very": "vˈɛɹi", "any": "ˈɛni", "every": "ˈɛvɹi",
    "again": "ɐɡˈɛn", "because": "bɪkˈʌz", "should": "ʃˌʊd", "through": "θɹuː", "though": "ðˌoʊ",
    "thought": "θˈɔːt", "know": "nˈoʊ", "knew": "nˈuː", "great": "ɡɹˈeɪt", "where": "wˌɛɹ",
    "why": "wˌaɪ", "our": "ˌaʊɚ", "hour": "ˈaʊɚ", "eye": "ˈaɪ", "answer": "ˈænsɚ", "says": "sˈɛz",
    "want": "wˈɑːnt", "once": "wˈʌns", "often": "ˈɔfən", "friend": "fɹˈɛnd", "both": "bˈoʊθ",
    "me": "miː", "us": "ˌʌs", "our's": "ˌaʊɚz", "am": "æm", "being": "bˈiːɪŋ", "here": "hˈɪɹ",
    "new": "nˈuː", "year": "jˈɪɹ", "work": "wˈɜːk", "put": "pˈʊt", "pull": "pˈʊl", "full": "fˈʊl",
    "push": "pˈʊʃ", "woman": "wˈʊmən", "women": "wˈɪmɪn", "build": "bˈɪld", "busy": "bˈɪzi",
    "listen": "lˈɪsən", "island": "ˈaɪlənd", "ocean": "ˈoʊʃən", "machine": "məʃˈiːn",
    "model": "mˈɑːdəl", "language": "lˈæŋɡwɪdʒ", "weather": "wˈɛðɚ", "together": "təɡˈɛðɚ",
    "little": "lˈɪɾəl", "mother": "mˈʌðɚ", "father": "fˈɑːðɚ", "brother": "bɹˈʌðɚ",
    "hundred": "hˈʌndɹɪd", "beautiful": "bjˈuːɾɪfəl", "around": "ɐɹˈaʊnd", "above": "ɐbˈʌv",
    "away": "ɐwˈeɪ", "alone": "ɐlˈoʊn", "across": "ɐkɹˈɔs", "today": "tədˈeɪ", "tomorrow": "təmˈɑːɹoʊ", "okay": "ˌoʊkˈeɪ", "ok": "ˌoʊkˈeɪ",
}

_ONES = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten",
         "eleven", "twelve", "thirteen", "fourteen", "fifteen", "sixteen", "seventeen", "eighteen",
         "nineteen"]
_TENS = ["", "", "twenty", "thirty", "forty", "fifty", "sixty", "seventy", "eighty", "ninety"]


def number_words(n: int) -> str:
    """Cardinal in words (espeak-ng reads digits as the number)."""
    if n < 0:
        return "minus " + number_words(-n)
    if n < 20:
        return _ONES[n]
    if n < 100:
        return _TENS[n // 10] + ("" if n % 10 == 0 else " " + _ONES[n % 10])
    if n < 1000:
        rest = n % 100
        return _ONES[n // 100] + " hundred" + ("" if rest == 0 else " and " + number_words(rest))
    for div, name in ((10 ** 9, "billion"), (10 ** 6, "million"), (1000, "thousand")):
        if n >= div:
            rest = n % div
            return number_words(n // div) + " " + name + ("" if rest == 0 else
                                                         (" and " if rest < 100 else " ") + number_words(rest))
    return str(n)


_SYMBOLS = {"&": " and ", "%": " percent ", "+": " plus ", "=": " equals ", "@": " at ", "$": " dollars "}


def normalize(text: str) -> str:
    text = text.replace("’", "'").replace("‘", "'").replace("“", '"').replace("”", '"')
    for k, v in _SYMBOLS.items():
        text = text.replace(k, v)
    text = re.sub(r"\d+", lambda m: " " + number_words(int(m.group(0))) + " ", text)
    return re.sub(r"[ \t]+", " ", text).strip()


# ---------------------------------------------------------------- letter-to-sound rules
_V = "aeiouy"
_IPA_VOWELS = ("aɪ", "aʊ", "eɪ", "oʊ", "ɔɪ", "iː", "uː", "ɑː", "ɔː", "ɜː", "oː",
               "æ", "ɛ", "ɪ", "ʌ", "ʊ", "ə", "ɚ", "ɐ", "i", "ɑ", "ɔ", "u", "e", "o", "a")

# (grapheme, phoneme, condition) -- tried longest grapheme first at each position; condition is
# None or a callable(word, i, j) on the grapheme span [i, j)
_MAGIC = {"a": "eɪ", "e": "iː", "i": "aɪ", "o": "oʊ", "u": "uː", "y": "aɪ"}
_SHORT = {"a": "æ", "e": "ɛ", "i": "ɪ", "o": "ɑː", "u": "ʌ", "y": "ɪ"}


def _is_v(c: str) -> bool:
    return c in _V


def _magic_e(w: str, i: int) -> bool:
    """w[i] is a vowel followed by one consonant and a silent final e (or e + s/d)."""
    j = i + 1
    if j >= len(w) or _is_v(w[j]) or w[j] in "wx":
        return False
    k = j + 1
    if w[j:j + 2] in ("th", "ch", "sh"):
        return w[j + 2:] == "e"   # bathe, ache; not fishes, riches
    tail = w[k:]
    return tail in ("e", "es", "ed", "er", "ers", "ely", "ement") and (w[j] != "r" or tail == "e")


_MULTI = [
    ("tion", "ʃən"), ("sion", "ʒən"), ("cial", "ʃəl"), ("tial", "ʃəl"), ("ture", "tʃɚ"), ("sure", "ʒɚ"),
    ("sch", "sk"), ("chr", "kɹ"), ("ough", "ʌf"), ("augh", "ɔː"), ("eigh", "eɪ"), ("igh", "aɪ"), ("tch", "tʃ"), ("dge", "dʒ"),
    ("air", "ɛɹ"), ("ear", "ɪɹ"), ("eer", "ɪɹ"), ("our", "aʊɚ"), ("ire", "aɪɚ"), ("are", "ɛɹ"),
    ("ore", "ɔːɹ"), ("ure", "jʊɹ"), ("ing", "ɪŋ"), ("ck", "k"), ("ch", "tʃ"), ("sh", "ʃ"), ("th", "θ"),
    ("ph", "f"), ("wh", "w"), ("ng", "ŋ"), ("qu", "kw"), ("gh", ""), ("ee", "iː"), ("ea", "iː"),
    ("ai", "eɪ"), ("ay", "eɪ"), ("ei", "eɪ"), ("ey", "eɪ"), ("oa", "oʊ"), ("oe", "oʊ"), ("oo", "uː"),
    ("ou", "aʊ"), ("oi", "ɔɪ"), ("oy", "ɔɪ"), ("au", "ɔː"), ("aw", "ɔː"), ("ew", "uː"), ("ue", "uː"),
    ("ui", "uː"), ("ie", "iː"), ("ar", "ɑːɹ"), ("or", "ɔːɹ"), ("er", "ɜː"), ("ir", "ɜː"), ("ur", "ɜː"),
    ("yr", "ɜː"),
]
_SINGLE = {"b": "b", "c": "k", "d": "d", "f": "f", "g": "ɡ", "h": "h", "j": "dʒ", "k": "k", "l": "l",
           "m": "m", "n": "n", "p": "p", "q": "k", "r": "ɹ", "s": "s", "t": "t", "v": "v", "w": "w",
           "x": "ks", "z": "z"}


def _letters(w: str) -> List[str]:
    """Grapheme -> phoneme units of one lower-case word (no stress yet)."""
    out: List[str] = []
    n = len(w)
    i = 0
    # silent initial letters
    if w.startswith(("kn", "gn", "wr", "pn", "ps")):
        i = 1
    while i < n:
        c = w[i]
        rest = w[i:]
        # final silent e (word has another vowel before it)
        if c == "e" and i == n - 1 and any(_is_v(x) for x in w[:i]) and not w.endswith(("ee", "ye")):
            if i >= 2 and w[i - 1] == "l" and not _is_v(w[i - 2]):
                out[-1:] = ["ə", "l"]   # -ble, -tle: syllabic l
            i += 1
            continue
        if rest == "les" and i > 0 and not _is_v(w[i - 1]):
            out.append("əlz")   # apples, tables
            i += 3
            continue
        if rest == "dges":
            out.append("dʒɪz")
            i += 4
            continue
        if (c == "e" and rest in ("es", "ed") and i > 1 and any(_is_v(x) for x in w[:i - 1])
                and not (w[i - 1] == "r" and not _is_v(w[i - 2]))):   # hundred, kindred: not a suffix
            prev = w[i - 1]
            sib = prev in "sxzj" or w[i - 2:i] in ("ch", "sh") or (prev in "cg" and i >= 2)
            unvoiced = prev in "pkfc" or w[i - 2:i] in ("ch", "sh") or prev == "s" or prev == "x"
            if rest == "ed":
                out.append("ɪd" if prev in "td" else ("t" if unvoiced else "d"))
            else:
                out.append("ɪz" if sib else ("s" if prev in "ptkf" else "z"))
            i += 2
            continue
        if c == "y" and i == 0:
            out.append("j")
            i += 1
            continue
        if c == "y" and i == n - 1 and i > 0:
            nv = sum(1 for x in w[:i] if _is_v(x))
            out.append("aɪ" if nv == 0 else "i")
            i += 1
            continue
        if c == "m" and rest == "mb":
            out.append("m")
            i += 2
            continue
        hit = None
        for g, p in _MULTI:
            if rest.startswith(g):
                # r-colour only before a consonant or the end ("ar" in "arid" is a + r)
                if g in ("ar", "or", "er", "ir", "ur", "yr") and len(rest) > 2 and _is_v(rest[2]):
                    continue
                if g in ("are", "ore", "ire", "ure") and len(rest) > 3:
                    continue
                if g == "gh" and i == 0:
                    p = "ɡ"
                if g == "th" and i == 0 and w in ("than", "thus", "though"):
                    p = "ð"
                if g == "ea" and rest.startswith("ead") and len(rest) <= 4:
                    p = "ɛ"   # head, dead, bread
                if g == "oo" and (rest.startswith("ook") or rest.startswith("ood")):
                    p = "ʊ"
                if g == "ou" and rest.startswith("ould"):
                    p = "ʊ"
                hit = (g, p)
                break
        if hit is None and rest.startswith("ow"):
            hit = ("ow", "oʊ" if i + 2 == n else "aʊ")
        if hit is not None:
            out.append(hit[1])
            i += len(hit[0])
            continue
        if _is_v(c):
            if c in "aou" and w[i + 1:i + 5] in ("tion", "sion"):
                out.append({"a": "eɪ", "o": "oʊ", "u": "uː"}[c])   # nation, motion, solution
            elif c != "y" and _magic_e(w, i):
                out.append(_MAGIC[c] if c != "u" or (i > 0 and w[i - 1] in "rlj") else "juː")
            elif c == "o" and i + 1 < n and w[i + 1] == "l" and (i + 2 == n or not _is_v(w[i + 2])):
                out.append("oʊ")   # old, bolt, cold
            elif c == "a" and i + 1 < n and w[i + 1] == "l" and (i + 2 == n or w[i + 2] in "lkt"):
                out.append("ɔː")   # all, talk, salt
            elif c == "i" and w[i + 1:i + 3] in ("nd", "ld"):
                out.append("aɪ")   # find, mild
            elif i == n - 1 and c in "eo":
                out.append("iː" if c == "e" else "oʊ")   # be, go
            elif i == n - 1 and c == "a":
                out.append("ə")
            elif c == "a" and i + 1 < n and w[i + 1] == "w":
                out.append("ɔː")
            else:
                out.append(_SHORT[c])
            i += 1
            continue
        # consonants
        nxt = w[i + 1] if i + 1 < n else ""
        if c == "s" and nxt == "c" and w[i + 2:i + 3] in ("e", "i", "y") and w[i + 2:i + 3]:
            out.append("s")   # science, scene: silent c
            i += 2
            continue
        if c == nxt and c not in "aeiou":
            i += 1   # doubled consonant: one phoneme
            continue
        if c == "c":
            out.append("s" if nxt and nxt in "eiy" else "k")
        elif c == "g":
            out.append("dʒ" if nxt and nxt in "eiy" and not w.startswith(("get", "give", "gift", "girl")) else "ɡ")
        elif c == "s":
            prev = w[i - 1] if i else ""
            voiced = (i == n - 1 and prev and prev not in "ptkfc") or (prev and _is_v(prev) and nxt and _is_v(nxt))
            out.append("z" if voiced else "s")
        elif c == "x" and i == 0:
            out.append("z")
        else:
            out.append(_SINGLE.get(c, ""))
        i += 1
    return [u for u in out if u]


_UNSTRESSED_PREFIX = ("be", "de", "re", "con", "com", "ex", "dis", "mis")
_PRE_STRESS_SUFFIX = ("tion", "sion", "ic", "ical", "ity", "ian", "ious", "eous", "ial", "ual")


_ATOM = re.compile("|".join(sorted(_IPA_VOWELS, key=len, reverse=True)) + "|tʃ|dʒ|.")


def _atoms(units: List[str]) -> List[str]:
    """Rule outputs ("ʃən", "ɑːɹ") -> single phonemes (vowels with their length mark)."""
    return _ATOM.findall("".join(units))


def _vowel_units(units: List[str]) -> List[int]:
    return [k for k, u in enumerate(units) if u in _IPA_VOWELS]


def _stress(word: str, units: List[str]) -> List[str]:
    vs = _vowel_units(units)
    if not vs:
        return units
    target = 0
    if len(vs) >= 2:
        if word.endswith(_PRE_STRESS_SUFFIX):
            target = len(vs) - 2
        elif word.startswith(_UNSTRESSED_PREFIX) and len(word) > 5 and not word.endswith(("er", "ing", "ly")):
            target = 1
    s = vs[target]
    out = list(units)
    # unstressed short vowels reduce (espeak-ng en-us: "banana" bɐnˈænə, "computer" kəm...)
    for k in vs:
        if k == s:
            continue
        u = out[k]
        if u in ("æ", "ʌ", "ɑː") and len(vs) > 1:
            out[k] = "ə"
        elif u == "ɛ" and 0 < k < len(out) - 1:
            out[k] = "ɪ"
        elif u == "ɜː":
            out[k] = "ɚ"
        elif u in ("ɔː", "ɑː") and k + 1 < len(out) and out[k + 1] == "ɹ":
            out[k] = "ɚ"   # unstressed -or / -ar: "information" ɪnfɚm..., "doctor"
            out[k + 1] = ""
    # en-us flap: t / d between the stressed vowel and an unstressed one
    for k in range(1, len(out) - 1):
        if out[k] in ("t", "d") and k - 1 == s and (k + 1) in vs and (k + 1) != s and out[k + 1] in ("ɚ", "ə", "i", "ɪ"):
            out[k] = "ɾ"
    out[s] = "ˈ" + out[s]
    return [u for u in out if u]


def word_ipa(word: str) -> str:
    w = word.lower()
    if w in LEXICON:
        return LEXICON[w]
    if w.endswith("'s") and w[:-2] in LEXICON:
        base = LEXICON[w[:-2]]
        return base + ("z" if base[-1] not in "sʃtkpf" else "s")
    w = w.replace("'", "")
    if not w:
        return ""
    if not any(_is_v(c) for c in w):   # an acronym / consonant cluster: spell it
        return " ".join(word_ipa(_LETTER_NAMES.get(c, c)) for c in w)
    return "".join(_stress(w, _atoms(_letters(w))))


_LETTER_NAMES = {"b": "bee", "c": "see", "d": "dee", "f": "ef", "g": "gee", "h": "aitch", "j": "jay",
                 "k": "kay", "l": "el", "m": "em", "n": "en", "p": "pee", "q": "queue", "r": "ar",
                 "s": "ess", "t": "tee", "v": "vee", "w": "double you", "x": "ex", "z": "zee"}
_TOKEN = re.compile(r"[A-Za-z']+|[.,!?;:\-()\"]")


def phonemize(text: str) -> str:
    """One sentence of English -> espeak-ng style IPA string (words separated by spaces,
    punctuation kept, e.g. "Hello world!" -> "həlˈoʊ wˈɜːld!")."""
    parts: List[str] = []
    for tok in _TOKEN.findall(normalize(text)):
        if tok[0].isalpha() or tok[0] == "'":
            ipa = word_ipa(tok)
            if ipa:
                parts.append(" " + ipa if parts else ipa)
        else:
            parts.append(tok if tok != "-" else " ")
    return "".join(parts).strip()


# phonemes a voice may lack, folded onto ones espeak voices generally have
_FOLD = {"ɚ": ["ə", "ɹ"], "ɜ": ["ə"], "ɐ": ["ə"], "ɾ": ["t"], "ᵻ": ["ɪ"], "ɡ": ["g"], "ɹ": ["r"],
         "ː": [], "ˌ": [], "ˈ": [], "ɑ": ["a"], "ɔ": ["o"], "ʊ": ["u"], "ɪ": ["i"], "ɛ": ["e"], "ʌ": ["ə"],
         "æ": ["a"], "θ": ["t"], "ð": ["d"], "ʃ": ["s"], "ʒ": ["z"], "ŋ": ["n"]}


def fold(phonemes: List[str], inventory) -> List[str]:
    """Map every phoneme outside `inventory` onto ones inside it (espeak -> a voice's map)."""
    out: List[str] = []
    for p in phonemes:
        if p in inventory:
            out.append(p)
            continue
        stack = list(_FOLD.get(p, []))
        while stack:
            q = stack.pop(0)
            if q in inventory:
                out.append(q)
            else:
                stack = list(_FOLD.get(q, [])) + stack
    return out
