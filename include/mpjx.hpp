// mpjx.hpp — C++ host mirror of the reference's mpiJava-1.2 reduction API over the C ABI (mpjx.h).
//
// Same names, argument meaning and error behaviour as the Java classes on this path:
//   mpi::MPI::SUM / MPI::DOUBLE ...           src/mpi/MPI.java:117-126, src/mpi/Datatype.java:57-66
//   mpi::Intracomm::Reduce(sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op, root)
//                                            src/mpi/Intracomm.java:740-760
//   ::Allreduce / ::Reduce_scatter / ::Scan / ::Bcast / ::Barrier
//                                            src/mpi/Intracomm.java:787-885
//   mpi::MPIException                        src/mpi/MPIException.java:42 (unchecked, like the Java one)
//   mpi::MPI::isOldSelected                  conf mpjexpress.mpi.old.collectives (src/mpi/MPI.java:70,266)
// Buffers are typed pointers; offsets and counts are in elements. Device pointers take the device
// path (blocking, like the Java calls); std::vector overloads are the host-resident path (the Java
// heap array case). Header-only: link libmpjx.
#pragma once
#include <mpjx.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace mpi {

class MPIException : public std::runtime_error {
 public:
  explicit MPIException(const std::string& m) : std::runtime_error(m) {}
};

inline void check(int status, const char* what) {
  if (status != MPJX_SUCCESS)
    throw MPIException(std::string(what) + ": " + mpjx_strerror(status) + ": " + mpjx_last_error());
}

// A basic type, or a (value, index) pair type SHORT2..DOUBLE2 = Contiguous(2, base)
// (src/mpi/MPI.java:110-114): `code` crosses the C ABI; buffers are arrays of the base type,
// offsets are base-element indices, counts are datatype elements (pairs).
struct Datatype {
  int code;
  int byteSize;  // bytes of the base type
  const char* name;
  int size = 1;
  int Size() const { return size; }
};

struct Op {
  int opCode;
  const char* name;
};

struct MPI {
  static constexpr Datatype BYTE{MPJX_BYTE, 1, "BYTE"};
  static constexpr Datatype CHAR{MPJX_CHAR, 2, "CHAR"};
  static constexpr Datatype SHORT{MPJX_SHORT, 2, "SHORT"};
  static constexpr Datatype BOOLEAN{MPJX_BOOLEAN, 1, "BOOLEAN"};
  static constexpr Datatype INT{MPJX_INT, 4, "INT"};
  static constexpr Datatype LONG{MPJX_LONG, 8, "LONG"};
  static constexpr Datatype FLOAT{MPJX_FLOAT, 4, "FLOAT"};
  static constexpr Datatype DOUBLE{MPJX_DOUBLE, 8, "DOUBLE"};
  static constexpr Datatype SHORT2{MPJX_SHORT2, 2, "SHORT2", 2};
  static constexpr Datatype INT2{MPJX_INT2, 4, "INT2", 2};
  static constexpr Datatype LONG2{MPJX_LONG2, 8, "LONG2", 2};
  static constexpr Datatype FLOAT2{MPJX_FLOAT2, 4, "FLOAT2", 2};
  static constexpr Datatype DOUBLE2{MPJX_DOUBLE2, 8, "DOUBLE2", 2};
  static constexpr Op MAX{MPJX_MAX, "MAX"}, MIN{MPJX_MIN, "MIN"}, SUM{MPJX_SUM, "SUM"},
      PROD{MPJX_PROD, "PROD"}, LAND{MPJX_LAND, "LAND"}, BAND{MPJX_BAND, "BAND"}, LOR{MPJX_LOR, "LOR"},
      BOR{MPJX_BOR, "BOR"}, LXOR{MPJX_LXOR, "LXOR"}, BXOR{MPJX_BXOR, "BXOR"}, MAXLOC{MPJX_MAXLOC, "MAXLOC"},
      MINLOC{MPJX_MINLOC, "MINLOC"};
  static inline bool isOldSelected = false;
};

// One rank's communicator (src/mpi/Intracomm.java). Not copyable; Free() or the destructor releases it.
class Intracomm {
 public:
  explicit Intracomm(mpjx_comm_t c, bool faithful = false) : c_(c), faithful_(faithful) {
    check(mpjx_comm_rank(c_, &rank_), "Rank");
    check(mpjx_comm_size(c_, &size_), "Size");
  }
  Intracomm(const Intracomm&) = delete;
  Intracomm& operator=(const Intracomm&) = delete;
  Intracomm(Intracomm&& o) noexcept : c_(o.c_), rank_(o.rank_), size_(o.size_), faithful_(o.faithful_) { o.c_ = nullptr; }
  ~Intracomm() { Free(); }

  int Rank() const { return rank_; }
  int Size() const { return size_; }
  mpjx_comm_t handle() const { return c_; }
  void Free() {
    if (c_) mpjx_comm_destroy(c_);
    c_ = nullptr;
  }
  void Barrier() { check(mpjx_barrier(c_), "Barrier"); }

  // ---- device-resident buffers (blocking) ----
  template <class T>
  void Reduce(const T* sendbuf, int sendoffset, T* recvbuf, int recvoffset, int count, const Datatype& dt,
              const Op& op, int root) {
    size_ok<T>(dt);
    // recvbuf: significant at the root; under faithful mode every rank's is written (MST partials)
    check(mpjx_reduce(c_, sendbuf + sendoffset, (rank_ == root || faithful_) ? recvbuf + recvoffset : nullptr, count,
                      dt.code, op.opCode, root, flags(), nullptr),
          "Reduce");
    sync();
  }
  template <class T>
  void Allreduce(const T* sendbuf, int sendoffset, T* recvbuf, int recvoffset, int count, const Datatype& dt,
                 const Op& op) {
    size_ok<T>(dt);
    check(mpjx_allreduce(c_, sendbuf + sendoffset, recvbuf + recvoffset, count, dt.code, op.opCode, flags(),
                         nullptr),
          "Allreduce");
    sync();
  }
  template <class T>
  void Reduce_scatter(const T* sendbuf, int sendoffset, T* recvbuf, int recvoffset, const std::vector<int>& recvcounts,
                      const Datatype& dt, const Op& op) {
    size_ok<T>(dt);
    std::vector<int64_t> rc = counts(recvcounts);
    check(mpjx_reduce_scatter(c_, sendbuf + sendoffset, recvbuf + recvoffset, rc.data(), dt.code, op.opCode,
                              flags(), nullptr),
          "Reduce_scatter");
    sync();
  }
  template <class T>
  void Scan(const T* sendbuf, int sendoffset, T* recvbuf, int recvoffset, int count, const Datatype& dt, const Op& op) {
    size_ok<T>(dt);
    check(mpjx_scan(c_, sendbuf + sendoffset, recvbuf + recvoffset, count, dt.code, op.opCode, flags(), nullptr),
          "Scan");
    sync();
  }
  template <class T>
  void Bcast(T* buf, int offset, int count, const Datatype& dt, int root) {
    size_ok<T>(dt);
    check(mpjx_bcast(c_, buf + offset, count, dt.code, root, nullptr), "Bcast");
    sync();
  }

  template <class T>
  void Gather(const T* sendbuf, int sendoffset, int sendcount, T* recvbuf, int recvoffset, int recvcount,
              const Datatype& dt, int root) {
    size_ok<T>(dt);
    if (sendcount != recvcount) throw MPIException("Gather: sendcount must equal recvcount");
    check(mpjx_gather(c_, sendbuf + sendoffset, rank_ == root ? recvbuf + recvoffset : nullptr, sendcount, dt.code,
                      root, nullptr),
          "Gather");
    sync();
  }
  template <class T>
  void Scatter(const T* sendbuf, int sendoffset, int sendcount, T* recvbuf, int recvoffset, int recvcount,
               const Datatype& dt, int root) {
    size_ok<T>(dt);
    if (sendcount != recvcount) throw MPIException("Scatter: sendcount must equal recvcount");
    check(mpjx_scatter(c_, rank_ == root ? sendbuf + sendoffset : nullptr, recvbuf + recvoffset, recvcount, dt.code,
                       root, nullptr),
          "Scatter");
    sync();
  }

  // ---- host-resident arrays (the Java heap array case) ----
  template <class T>
  void Reduce(const std::vector<T>& sendbuf, int sendoffset, std::vector<T>& recvbuf, int recvoffset, int count,
              const Datatype& dt, const Op& op, int root) {
    size_ok<T>(dt);
    extent(sendbuf, sendoffset, count, dt.Size());
    const bool all_recv = rank_ == root || faithful_;  // faithful: every rank's recvbuf is written
    if (all_recv) extent(recvbuf, recvoffset, count, dt.Size());
    check(mpjx_reduce_host(c_, sendbuf.data() + sendoffset, all_recv ? recvbuf.data() + recvoffset : nullptr,
                           count, dt.code, op.opCode, root, flags()),
          "Reduce");
  }
  template <class T>
  void Allreduce(const std::vector<T>& sendbuf, int sendoffset, std::vector<T>& recvbuf, int recvoffset, int count,
                 const Datatype& dt, const Op& op) {
    size_ok<T>(dt);
    extent(sendbuf, sendoffset, count, dt.Size());
    extent(recvbuf, recvoffset, count, dt.Size());
    check(mpjx_allreduce_host(c_, sendbuf.data() + sendoffset, recvbuf.data() + recvoffset, count, dt.code,
                              op.opCode, flags()),
          "Allreduce");
  }
  template <class T>
  void Reduce_scatter(const std::vector<T>& sendbuf, int sendoffset, std::vector<T>& recvbuf, int recvoffset,
                      const std::vector<int>& recvcounts, const Datatype& dt, const Op& op) {
    size_ok<T>(dt);
    std::vector<int64_t> rc = counts(recvcounts);
    int64_t total = 0;
    for (int64_t x : rc) total += x;
    extent(sendbuf, sendoffset, total, dt.Size());
    extent(recvbuf, recvoffset, rc[rank_], dt.Size());
    check(mpjx_reduce_scatter_host(c_, sendbuf.data() + sendoffset, recvbuf.data() + recvoffset, rc.data(),
                                   dt.code, op.opCode, flags()),
          "Reduce_scatter");
  }
  template <class T>
  void Scan(const std::vector<T>& sendbuf, int sendoffset, std::vector<T>& recvbuf, int recvoffset, int count,
            const Datatype& dt, const Op& op) {
    size_ok<T>(dt);
    extent(sendbuf, sendoffset, count, dt.Size());
    extent(recvbuf, recvoffset, count, dt.Size());
    check(mpjx_scan_host(c_, sendbuf.data() + sendoffset, recvbuf.data() + recvoffset, count, dt.code,
                         op.opCode, flags()),
          "Scan");
  }

 private:
  // the mpiJava calls are blocking: every call returns complete (MPJX_FLAG_BLOCKING)
  unsigned flags() const {
    return (MPI::isOldSelected ? MPJX_FLAG_OLD_COLLECTIVES : 0u) | (faithful_ ? MPJX_FLAG_FAITHFUL : 0u) |
           MPJX_FLAG_BLOCKING;
  }
  void sync() { check(mpjx_comm_synchronize(c_), "synchronize"); }
  template <class T>
  static void size_ok(const Datatype& dt) {
    if ((int)sizeof(T) != dt.byteSize)
      throw MPIException(std::string("buffer element size does not match MPI.") + dt.name);
  }
  template <class T>
  static void extent(const std::vector<T>& v, int off, int64_t count, int size = 1) {
    if (off < 0 || count < 0 || (int64_t)off + count * size > (int64_t)v.size())
      throw MPIException("offset + count exceeds the array length");
  }
  std::vector<int64_t> counts(const std::vector<int>& rc) const {
    if ((int)rc.size() < size_) throw MPIException("recvcounts shorter than the communicator");
    return std::vector<int64_t>(rc.begin(), rc.begin() + size_);
  }

  mpjx_comm_t c_;
  int rank_ = 0, size_ = 1;
  bool faithful_;
};

// Multicore mode (smpdev): nranks ranks that are threads of this process, all on `devices`.
inline std::vector<Intracomm> smp_world(int nranks, const std::vector<int>& devices) {
  std::vector<mpjx_comm_t> h(nranks);
  check(mpjx_comm_init_smp(h.data(), nranks, devices.data()), "mpjx_comm_init_smp");
  std::vector<Intracomm> w;
  w.reserve(nranks);
  for (mpjx_comm_t c : h) w.emplace_back(c);
  return w;
}

// One process per GPU over RCCL (MPJDev.init + COMM_WORLD, src/mpi/MPI.java:298-305): every rank
// passes the id rank 0 got from mpjx_get_unique_id, shared out of band.
inline Intracomm Init(int rank, int size, int device, const mpjx_unique_id& id) {
  mpjx_comm_t c = nullptr;
  check(mpjx_comm_init_rank(&c, size, &id, rank, device), "mpjx_comm_init_rank");
  return Intracomm(c);
}

// Processes of one node without RCCL: the HIP-IPC direct engine (id: any bytes unique to the world).
inline Intracomm InitIPC(int rank, int size, int device, const mpjx_unique_id& id) {
  mpjx_comm_t c = nullptr;
  check(mpjx_comm_init_ipc(&c, size, &id, rank, device), "mpjx_comm_init_ipc");
  return Intracomm(c);
}

// Multicore mode, formed by the rank threads themselves (each thread calls this for its rank with the
// world's id and all ranks' devices; one world per communicator, as Split/Create need).
inline Intracomm InitSMPRank(int rank, int size, const std::vector<int>& devices, const mpjx_unique_id& id) {
  mpjx_comm_t c = nullptr;
  check(mpjx_comm_init_smp_rank(&c, size, &id, rank, devices.data()), "mpjx_comm_init_smp_rank");
  return Intracomm(c);
}

}  // namespace mpi
