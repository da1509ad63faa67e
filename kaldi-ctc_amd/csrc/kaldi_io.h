// kaldi_io.h -- the Kaldi token stream in both modes (model files).
//
//   WriteToken / ReadToken / ExpectToken      base/io-funcs.cc (token + one space, both modes)
//   WriteBasicType / ReadBasicType           base/io-funcs-inl.h (binary: size byte + raw
//                                            little-endian value; bool: 'T' / 'F')
//   WriteIntegerVector / ReadIntegerVector   base/io-funcs-inl.h (binary: size byte, int32
//                                            count, raw elements; text "[ a b ]")
//   Vector<float>::Write / Read              matrix/kaldi-vector.cc ("FV" n raw | " [ a b ]")
//   Matrix<float>::Write / Read              matrix/kaldi-matrix.cc ("FM" rows cols raw |
//                                            " [\n  a b \n  c d ]")
//   InitKaldiOutputStream / InitKaldiInputStream  base/io-funcs.cc ("\0B" binary header)
// Text floats are written with 9 significant digits (exact round trip).
#pragma once
#include <cctype>
#include <cstdint>
#include <cstring>
#include <iomanip>
#include <istream>
#include <limits>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

namespace kctc {
namespace kio {

[[noreturn]] inline void Fail(const std::string &what) { throw std::runtime_error("Kaldi I/O: " + what); }

// "\0B" on a binary stream; returns whether the stream is binary.
inline void InitOutput(std::ostream &os, bool binary) {
  if (binary) {
    os.put('\0');
    os.put('B');
  }
}
inline bool InitInput(std::istream &is) {
  if (is.peek() == '\0') {
    is.get();
    if (is.peek() != 'B') Fail("bad binary header");
    is.get();
    return true;
  }
  return false;
}

inline void WriteToken(std::ostream &os, bool, const std::string &t) {
  if (t.empty() || t.find(' ') != std::string::npos) Fail("bad token '" + t + "'");
  os << t << ' ';
}
inline std::string ReadToken(std::istream &is, bool binary) {
  if (!binary) is >> std::ws;
  std::string s;
  is >> s;
  if (is.fail()) Fail("ReadToken failed");
  if (!isspace(is.peek())) Fail("expected a space after token " + s);
  is.get();
  return s;
}
inline void ExpectToken(std::istream &is, bool binary, const std::string &t) {
  const std::string s = ReadToken(is, binary);
  if (s != t) Fail("expected token " + t + ", got " + s);
}
inline std::string PeekToken(std::istream &is, bool binary) {
  const auto pos = is.tellg();
  std::string s = ReadToken(is, binary);
  is.seekg(pos);
  return s;
}

inline void WriteInt(std::ostream &os, bool binary, int32_t v) {
  if (binary) {
    os.put((char)sizeof(v));
    os.write(reinterpret_cast<const char *>(&v), sizeof(v));
  } else {
    os << v << ' ';
  }
}
inline int32_t ReadInt(std::istream &is, bool binary) {
  if (binary) {
    const int c = is.get();
    if (c != (int)sizeof(int32_t)) Fail("ReadBasicType<int32>: size byte " + std::to_string(c));
    int32_t v;
    is.read(reinterpret_cast<char *>(&v), sizeof(v));
    if (!is) Fail("ReadBasicType<int32>: truncated");
    return v;
  }
  long long v;
  is >> v;
  if (is.fail()) Fail("ReadBasicType<int32>: not an integer");
  return (int32_t)v;
}
inline void WriteFloat(std::ostream &os, bool binary, float v) {
  if (binary) {
    os.put((char)sizeof(v));
    os.write(reinterpret_cast<const char *>(&v), sizeof(v));
  } else {
    os << std::setprecision(7) << v << ' ';
  }
}
inline float ReadFloat(std::istream &is, bool binary) {
  if (binary) {
    const int c = is.get();
    if (c == 4) {
      float v;
      is.read(reinterpret_cast<char *>(&v), 4);
      if (!is) Fail("ReadBasicType<float>: truncated");
      return v;
    }
    if (c == 8) {  // written as double (ReadBasicType<float> accepts both)
      double v;
      is.read(reinterpret_cast<char *>(&v), 8);
      if (!is) Fail("ReadBasicType<float>: truncated");
      return (float)v;
    }
    Fail("ReadBasicType<float>: size byte " + std::to_string(c));
  }
  double v;
  is >> v;
  if (is.fail()) Fail("ReadBasicType<float>: not a number");
  return (float)v;
}
inline void WriteDouble(std::ostream &os, bool binary, double v) {
  if (binary) {
    os.put((char)sizeof(v));
    os.write(reinterpret_cast<const char *>(&v), sizeof(v));
  } else {
    os << std::setprecision(7) << v << ' ';
  }
}
inline double ReadDouble(std::istream &is, bool binary) {
  if (binary) {
    const int c = is.get();
    if (c == 8) {
      double v;
      is.read(reinterpret_cast<char *>(&v), 8);
      if (!is) Fail("ReadBasicType<double>: truncated");
      return v;
    }
    if (c == 4) {
      float v;
      is.read(reinterpret_cast<char *>(&v), 4);
      if (!is) Fail("ReadBasicType<double>: truncated");
      return v;
    }
    Fail("ReadBasicType<double>: size byte " + std::to_string(c));
  }
  double v;
  is >> v;
  if (is.fail()) Fail("ReadBasicType<double>: not a number");
  return v;
}
inline void WriteBool(std::ostream &os, bool binary, bool b) {
  os << (b ? "T" : "F");
  if (!binary) os << ' ';
}
inline bool ReadBool(std::istream &is, bool binary) {
  if (!binary) is >> std::ws;
  const int c = is.peek();
  if (c == 'T' || c == 'F') {
    is.get();
    return c == 'T';
  }
  Fail("ReadBasicType<bool>: expected T or F");
}

inline void WriteIntVector(std::ostream &os, bool binary, const std::vector<int32_t> &v) {
  if (binary) {
    os.put((char)sizeof(int32_t));
    const int32_t n = (int32_t)v.size();
    os.write(reinterpret_cast<const char *>(&n), 4);
    if (n) os.write(reinterpret_cast<const char *>(v.data()), 4 * (size_t)n);
  } else {
    os << "[ ";
    for (int32_t x : v) os << x << ' ';
    os << "]\n";
  }
}
inline std::vector<int32_t> ReadIntVector(std::istream &is, bool binary) {
  std::vector<int32_t> v;
  if (binary) {
    if (is.get() != (int)sizeof(int32_t)) Fail("ReadIntegerVector: size byte");
    int32_t n;
    is.read(reinterpret_cast<char *>(&n), 4);
    if (!is || n < 0) Fail("ReadIntegerVector: bad size");
    v.resize(n);
    if (n) is.read(reinterpret_cast<char *>(v.data()), 4 * (size_t)n);
    if (!is) Fail("ReadIntegerVector: truncated");
    return v;
  }
  std::string s;
  is >> s;
  if (s != "[") Fail("ReadIntegerVector: expected [");
  while (is >> s && s != "]") v.push_back(std::stoi(s));
  if (s != "]") Fail("ReadIntegerVector: expected ]");
  return v;
}

inline void WriteFloatVector(std::ostream &os, bool binary, const float *v, long n) {
  if (binary) {
    WriteToken(os, binary, "FV");
    WriteInt(os, binary, (int32_t)n);
    if (n) os.write(reinterpret_cast<const char *>(v), 4 * (size_t)n);
  } else {
    os << " [ ";
    for (long i = 0; i < n; i++) os << std::setprecision(7) << v[i] << ' ';
    os << "]\n";
  }
}
inline std::vector<float> ReadFloatVector(std::istream &is, bool binary) {
  std::vector<float> v;
  if (binary) {
    const std::string t = ReadToken(is, binary);
    const int32_t n = ReadInt(is, binary);
    if (n < 0) Fail("Vector::Read: negative size");
    v.resize(n);
    if (t == "FV") {
      if (n) is.read(reinterpret_cast<char *>(v.data()), 4 * (size_t)n);
    } else if (t == "DV") {
      std::vector<double> d(n);
      if (n) is.read(reinterpret_cast<char *>(d.data()), 8 * (size_t)n);
      for (int32_t i = 0; i < n; i++) v[i] = (float)d[i];
    } else {
      Fail("Vector::Read: expected FV or DV, got " + t);
    }
    if (!is) Fail("Vector::Read: truncated");
    return v;
  }
  std::string s;
  is >> s;
  if (s != "[") Fail("Vector::Read: expected [, got " + s);
  while (is >> s && s != "]") v.push_back(std::stof(s));
  if (s != "]") Fail("Vector::Read: expected ]");
  return v;
}

// Vector<double>::Write / Read ("DV" n raw | " [ a b ]"); a float vector is accepted
inline void WriteDoubleVector(std::ostream &os, bool binary, const std::vector<double> &v) {
  if (binary) {
    WriteToken(os, binary, "DV");
    WriteInt(os, binary, (int32_t)v.size());
    if (!v.empty()) os.write(reinterpret_cast<const char *>(v.data()), 8 * v.size());
  } else {
    os << " [ ";
    for (double x : v) os << std::setprecision(7) << x << ' ';
    os << "]\n";
  }
}
inline std::vector<double> ReadDoubleVector(std::istream &is, bool binary) {
  std::vector<double> v;
  if (binary) {
    const std::string t = ReadToken(is, binary);
    const int32_t n = ReadInt(is, binary);
    if (n < 0) Fail("Vector::Read: negative size");
    v.resize(n);
    if (t == "DV") {
      if (n) is.read(reinterpret_cast<char *>(v.data()), 8 * (size_t)n);
    } else if (t == "FV") {
      std::vector<float> f(n);
      if (n) is.read(reinterpret_cast<char *>(f.data()), 4 * (size_t)n);
      for (int32_t i = 0; i < n; i++) v[i] = f[i];
    } else {
      Fail("Vector::Read: expected DV or FV, got " + t);
    }
    if (!is) Fail("Vector::Read: truncated");
    return v;
  }
  std::string s;
  is >> s;
  if (s != "[") Fail("Vector::Read: expected [, got " + s);
  while (is >> s && s != "]") v.push_back(std::stod(s));
  if (s != "]") Fail("Vector::Read: expected ]");
  return v;
}

inline void WriteFloatMatrix(std::ostream &os, bool binary, const float *m, int rows, int cols) {
  if (binary) {
    WriteToken(os, binary, "FM");
    WriteInt(os, binary, rows);
    WriteInt(os, binary, cols);
    if ((long)rows * cols) os.write(reinterpret_cast<const char *>(m), 4 * (size_t)rows * cols);
    return;
  }
  if (cols == 0) {
    os << " [ ]\n";
    return;
  }
  os << " [";
  for (int r = 0; r < rows; r++) {
    os << "\n  ";
    for (int c = 0; c < cols; c++) os << std::setprecision(7) << m[(size_t)r * cols + c] << ' ';
  }
  os << "]\n";
}
// row-major; *rows / *cols set
inline std::vector<float> ReadFloatMatrix(std::istream &is, bool binary, int *rows, int *cols) {
  std::vector<float> m;
  if (binary) {
    const std::string t = ReadToken(is, binary);
    *rows = ReadInt(is, binary);
    *cols = ReadInt(is, binary);
    if (*rows < 0 || *cols < 0) Fail("Matrix::Read: negative size");
    const size_t n = (size_t)*rows * *cols;
    m.resize(n);
    if (t == "FM") {
      if (n) is.read(reinterpret_cast<char *>(m.data()), 4 * n);
    } else if (t == "DM") {
      std::vector<double> d(n);
      if (n) is.read(reinterpret_cast<char *>(d.data()), 8 * n);
      for (size_t i = 0; i < n; i++) m[i] = (float)d[i];
    } else {
      Fail("Matrix::Read: expected FM or DM, got " + t);
    }
    if (!is) Fail("Matrix::Read: truncated");
    return m;
  }
  // text: "[", rows separated by newlines, "]"
  std::string s;
  is >> s;
  if (s != "[") Fail("Matrix::Read: expected [, got " + s);
  *rows = 0;
  *cols = 0;
  int in_row = 0;
  for (;;) {
    int c = is.peek();
    if (c == EOF) Fail("Matrix::Read: unterminated");
    if (c == '\n') {
      is.get();
      if (in_row) {
        if (*rows == 0) *cols = in_row;
        else if (in_row != *cols) Fail("Matrix::Read: ragged rows");
        (*rows)++;
        in_row = 0;
      }
      continue;
    }
    if (isspace(c)) {
      is.get();
      continue;
    }
    is >> s;
    if (s == "]") {
      if (in_row) {
        if (*rows == 0) *cols = in_row;
        else if (in_row != *cols) Fail("Matrix::Read: ragged rows");
        (*rows)++;
      }
      break;
    }
    m.push_back(std::stof(s));
    in_row++;
  }
  return m;
}

}  // namespace kio
}  // namespace kctc
