"""Vocabulary: the reference's ``dict.pkl`` read WITHOUT unpickling.

The reference loads ``(word2int, int2word)`` with ``pickle.load`` (data.py:373-374).
Executing a pickle that ships with a third-party repo is not acceptable here, so this
module walks the pickle opcode stream with :mod:`pickletools` (which never executes
anything) and rebuilds the two dicts with a tiny stack machine that only understands
the container/str/int opcodes.  Any other opcode (GLOBAL, REDUCE, BUILD, ...) is
rejected, so a malicious file cannot run code.

The parsed vocabulary is also committed as ``vocab.json`` next to the package so that
the GPU box (which has no ``/root/reference``) gets the identical table.
"""
import json
import os
import pickletools

_HERE = os.path.dirname(os.path.abspath(__file__))
VOCAB_JSON = os.path.join(os.path.dirname(_HERE), "vocab.json")

_MARK = object()


def _safe_unpickle(data):
    """Rebuild a pickle made only of dict/tuple/list/str/int/float/bool/None opcodes."""
    stack, memo = [], {}

    def pop_mark():
        items = []
        while True:
            x = stack.pop()
            if x is _MARK:
                break
            items.append(x)
        items.reverse()
        return items

    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        elif name == "STOP":
            break
        elif name in ("EMPTY_DICT",):
            stack.append({})
        elif name in ("EMPTY_LIST",):
            stack.append([])
        elif name in ("EMPTY_TUPLE",):
            stack.append(())
        elif name == "MARK":
            stack.append(_MARK)
        elif name in ("BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8", "UNICODE"):
            stack.append(str(arg))
        elif name in ("BININT", "BININT1", "BININT2", "INT", "LONG1", "LONG4", "LONG"):
            stack.append(int(arg))
        elif name in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif name == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif name == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif name == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif name == "TUPLE1":
            stack[-1:] = [tuple(stack[-1:])]
        elif name == "TUPLE2":
            stack[-2:] = [tuple(stack[-2:])]
        elif name == "TUPLE3":
            stack[-3:] = [tuple(stack[-3:])]
        else:
            raise ValueError(f"dict.pkl: opcode {name} is not allowed by the safe loader")
    if len(stack) != 1:
        raise ValueError("dict.pkl: malformed pickle stream")
    return stack[0]


def load_dict_pkl(path):
    """Return ``(word2int, int2word)`` from a reference ``dict.pkl`` (no code executed)."""
    with open(path, "rb") as f:
        data = f.read()
    obj = _safe_unpickle(data)
    if not (isinstance(obj, tuple) and len(obj) == 2):
        raise ValueError("dict.pkl must hold a (word2int, int2word) tuple")
    word2int, int2word = obj
    return dict(word2int), {int(k): v for k, v in int2word.items()}


def save_vocab_json(int2word, path=VOCAB_JSON):
    items = [int2word[i] for i in range(len(int2word))]
    with open(path, "w", encoding="utf-8") as f:
        json.dump(items, f, ensure_ascii=False, indent=0)


def load_vocab(path=None):
    """``(word2int, int2word)``: from ``path`` if given (a dict.pkl or vocab.json), else the
    committed ``vocab.json``."""
    path = path or VOCAB_JSON
    if path.endswith(".pkl"):
        return load_dict_pkl(path)
    with open(path, "r", encoding="utf-8") as f:
        items = json.load(f)
    int2word = {i: w for i, w in enumerate(items)}
    word2int = {w: i for i, w in int2word.items()}
    return word2int, int2word
