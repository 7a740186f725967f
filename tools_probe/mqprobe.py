import ctypes, os, resource
print("RLIMIT_MSGQUEUE", resource.getrlimit(resource.RLIMIT_MSGQUEUE), "NOFILE", resource.getrlimit(resource.RLIMIT_NOFILE))
for f in ("msg_max","msgsize_max","queues_max"):
    print(f, open(f"/proc/sys/fs/mqueue/{f}").read().strip())
rt = ctypes.CDLL("librt.so.1", use_errno=True)
class Attr(ctypes.Structure):
    _fields_=[("flags",ctypes.c_long),("maxmsg",ctypes.c_long),("msgsize",ctypes.c_long),("cur",ctypes.c_long),("pad",ctypes.c_long*4)]
rt.mq_open.restype=ctypes.c_int
for maxmsg in (8,4,2,1):
    a=Attr(0,maxmsg,160,0)
    name=f"/probe_{os.getpid()}_{maxmsg}".encode()
    fd=rt.mq_open(name, os.O_RDONLY|os.O_CREAT|os.O_EXCL, 0o600, ctypes.byref(a))
    print("maxmsg",maxmsg,"fd",fd,"errno",os.strerror(ctypes.get_errno()) if fd<0 else "")
    if fd>=0: rt.mq_unlink(name)
print("uid", os.getuid(), "user", os.environ.get("USER"))
