/*
 * HipIntracomm — the Java side of the MI355X reduction path (new code for a maintainer to add to
 * src/mpi; NOT compiled in this repository: the build image has no JDK).
 *
 * Mirrors how NativeIntracomm plugs into the reference (src/mpi/NativeIntracomm.java:42,1072-1115):
 * it extends PureIntracomm, overrides the four reductions, and falls back to super for everything
 * the GPU path does not cover — non-primitive or derived datatypes (baseType > 8, Size() > 1, except
 * MAXLOC/MINLOC on the pair types SHORT2..DOUBLE2, which the GPU path has), other user-defined ops
 * (op.worker == null), and buffers below a size threshold where PCIe staging would dominate. Selected in the Intracomm constructor
 * (src/mpi/Intracomm.java:63-67) when the device name passed to MPJDev.init is "hip"
 * (see INTEGRATION.md for the three-line patch).
 */
package mpi;

import mpjdev.Constants;

public class HipIntracomm extends PureIntracomm {

  static {
    System.loadLibrary("mpjx_jni");  // libmpjx_jni.so -> libmpjx.so
  }

  /* flags of include/mpjx.h */
  static final int FLAG_OLD_COLLECTIVES = 0x1;
  static final int FLAG_FAITHFUL = 0x2;

  /** Elements below which the pure-Java path stays cheaper than staging through the GPU. */
  static int THRESHOLD_BYTES = Integer.getInteger("mpjx.threshold.bytes", 1 << 20);

  private final long comm;  // mpjx_comm_t

  HipIntracomm(mpjdev.Comm mpjdevComm, mpi.Group group) throws MPIException {
    super(mpjdevComm, group);
    int rank = mpjdevComm.id(), size = mpjdevComm.size();
    int device = Integer.getInteger("mpjx.device", rank % Math.max(1, nativeDeviceCount()));
    if (Boolean.getBoolean("mpjx.multicore")) {
      // smpdev: ranks are threads of this JVM; the first thread creates every rank's communicator
      comm = nativeInitSmp(rank, size, device);
    } else {
      // one JVM per GPU: rank 0 makes the world id, the existing host Bcast hands it out; the engine
      // is RCCL's exchange (default) or the HIP-IPC direct engine (-Dmpjx.engine=ipc, JVMs of one node)
      byte[] uid = new byte[128];
      if (rank == 0) nativeUniqueId(uid);
      super.Bcast(uid, 0, 128, MPI.BYTE, 0);
      comm = "ipc".equals(System.getProperty("mpjx.engine", "rccl"))
          ? nativeInitIpc(rank, size, device, uid)
          : nativeInitRank(rank, size, device, uid);
    }
  }

  /** Typed ops 1..10 on basic types, or MAXLOC/MINLOC (11/12, User_function ops with an opCode,
   *  src/mpi/MPI.java:127-130) on the pair types SHORT2..DOUBLE2 (Contiguous(2, base)). */
  private static boolean gpuEligible(Datatype t, Op op, int count) {
    boolean typed = t.baseType >= 1 && t.baseType <= 8 && t.Size() == 1 && op.worker != null
        && op.opCode >= 1 && op.opCode <= 10;
    boolean loc = (op.opCode == 11 || op.opCode == 12) && t.Size() == 2
        && (t.baseType == 3 || (t.baseType >= 5 && t.baseType <= 8));
    return (typed || loc) && (long) count * t.Size() * t.byteSize >= THRESHOLD_BYTES;
  }

  /** C-ABI type code (include/mpjx.h): baseType, or 0x100 | baseType for the pair types. */
  private static int code(Datatype t) {
    return t.Size() == 2 ? (0x100 | t.baseType) : t.baseType;
  }

  private int flags() {
    return MPI.isOldSelected ? FLAG_OLD_COLLECTIVES : 0;
  }

  public void Reduce(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, int count,
      Datatype datatype, Op op, int root) throws MPIException {
    if (!gpuEligible(datatype, op, count)) {
      super.Reduce(sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op, root);
      return;
    }
    nativeReduce(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, root, flags());
  }

  public void Allreduce(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, int count,
      Datatype datatype, Op op) throws MPIException {
    if (!gpuEligible(datatype, op, count)) {
      super.Allreduce(sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op);
      return;
    }
    nativeAllreduce(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, flags());
  }

  public void Reduce_scatter(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset,
      int[] recvcounts, Datatype datatype, Op op) throws MPIException {
    int total = 0;
    for (int i = 0; i < Size(); i++) total += recvcounts[i];
    if (!gpuEligible(datatype, op, total)) {
      super.Reduce_scatter(sendbuf, sendoffset, recvbuf, recvoffset, recvcounts, datatype, op);
      return;
    }
    nativeReduceScatter(comm, sendbuf, sendoffset, recvbuf, recvoffset, recvcounts,
        code(datatype), op.opCode, flags());
  }

  public void Scan(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, int count,
      Datatype datatype, Op op) throws MPIException {
    if (!gpuEligible(datatype, op, count)) {
      super.Scan(sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op);
      return;
    }
    nativeScan(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, flags());
  }

  /* ---- JNI (integration/jni/mpi_HipIntracomm.c); failures throw mpi.MPIException ---- */
  private static native int nativeDeviceCount();
  private static native void nativeUniqueId(byte[] uid);
  private static native long nativeInitRank(int rank, int size, int device, byte[] uid);
  private static native long nativeInitSmp(int rank, int size, int device);
  private static native long nativeInitIpc(int rank, int size, int device, byte[] uid);
  private native void nativeReduce(long comm, Object send, int soff, Object recv, int roff,
      int count, int type, int op, int root, int flags);
  private native void nativeAllreduce(long comm, Object send, int soff, Object recv, int roff,
      int count, int type, int op, int flags);
  private native void nativeReduceScatter(long comm, Object send, int soff, Object recv, int roff,
      int[] recvcounts, int type, int op, int flags);
  private native void nativeScan(long comm, Object send, int soff, Object recv, int roff,
      int count, int type, int op, int flags);
}
