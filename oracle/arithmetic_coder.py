"""Pure-Python restatement of code/coding.pyx:27-216 (ArithmeticCoder.encode /
decode, linear symbol search).  TEST INFRASTRUCTURE ONLY -- the checker for
the C++ coder in libcwq.so; integer arithmetic, so exactly reproducible.
Parity with the Cython original is unpinned by fixtures (none ship with the
reference; coding_test.py is unseeded and broken at :30) and rests on this
line-by-line restatement (the reference may not be built here: SURVEY 8(c))."""


class ArithmeticCoderRef(object):
    def __init__(self, P, precision=32):
        self.precision = precision
        c = 0
        self.C, self.D = [], []
        for p in P:                       # :42-48
            self.C.append(c)
            c += int(p)
            self.D.append(c)
        self.R = c

    def encode(self, message):            # :59-125
        whole = 2 ** self.precision
        half = 2 ** (self.precision - 1)
        quarter = 2 ** (self.precision - 2)
        low, high, s = 0, whole, 0
        code = []
        for sym in message:
            width = high - low
            high = low + (width * self.D[sym]) // self.R
            low = low + (width * self.C[sym]) // self.R
            while high < half or low > half:
                if high < half:
                    code.extend("0" + "1" * s)
                    s = 0
                    low *= 2
                    high *= 2
                elif low > half:
                    code.extend("1" + "0" * s)
                    s = 0
                    low = (low - half) * 2
                    high = (high - half) * 2
            while low > quarter and high < 3 * quarter:
                s += 1
                low = (low - quarter) * 2
                high = (high - quarter) * 2
        s += 1
        if low <= quarter:
            code.extend("0" + "1" * s)
        else:
            code.extend("1" + "0" * s)
        return code

    def decode(self, code, max_symbols=10 ** 7):  # :129-216
        precision = self.precision
        whole = 2 ** precision
        half = 2 ** (precision - 1)
        quarter = 2 ** (precision - 2)
        low, high = 0, whole
        z, i = 0, 0
        while i < precision and i < len(code):
            if code[i] == '1':
                z += 2 ** (precision - i - 1)
            i += 1
        message = []
        while len(message) < max_symbols:
            for j in range(len(self.C)):
                width = high - low
                high_ = low + (width * self.D[j]) // self.R
                low_ = low + (width * self.C[j]) // self.R
                if low_ <= z < high_:
                    message.append(j)
                    high, low = high_, low_
                    if j == 0:
                        return message
                    while high < half or low > half:
                        if high < half:
                            low *= 2
                            high *= 2
                            z *= 2
                        elif low > half:
                            low = (low - half) * 2
                            high = (high - half) * 2
                            z = (z - half) * 2
                        if i < len(code) and code[i] == '1':
                            z += 1
                        i += 1
                    while low > quarter and high < 3 * quarter:
                        low = (low - quarter) * 2
                        high = (high - quarter) * 2
                        z = (z - quarter) * 2
                        if i < len(code) and code[i] == '1':
                            z += 1
                        i += 1
        raise RuntimeError("no EOF within max_symbols")
