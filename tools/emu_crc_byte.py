# CPU emulation of the JFSX_CRC_BYTE lane algorithm of jfsx_crc.hip (table layout, v_perm selectors,
# slice-by-4 chains, 4096-B span shift, lane-to-segment-end shift) against bytewise CRC32C.
# Standalone check: python3 tools/emu_crc_byte.py
import numpy as np, os
P=0x82F63B78
T=[0]*256
for i in range(256):
    c=i
    for _ in range(8): c=(c>>1)^P if c&1 else c>>1
    T[i]=c
def mulmod(a,b):  # reflected GF(2) multiply mod P (bit 31 = x^0)
    p=0
    for i in range(32):
        if a & (0x80000000>>i): p^=b
        b = (b>>1)^P if b&1 else b>>1
    return p
x8=[0x00800000]
for k in range(1,32): x8.append(mulmod(x8[-1],x8[-1]))
def xpow8(n):
    r=0x80000000;k=0
    while n:
        if n&1: r=mulmod(x8[k],r)
        n>>=1;k+=1
    return r
crc=[0]*(32*256)
for j in range(16):
    xp=xpow8(15-j)
    for b in range(256): crc[j*256+b]=mulmod(xp,T[b])
x4096=xpow8(4096)
for k in range(4):
    for v in range(256): crc[(28+k)*256+v]=mulmod(x4096, v<<(8*k))
lds=bytearray(0x24000)
import struct
for t in range(4):
    for e in range(256):
        for bank in range(32):
            struct.pack_into('<I',lds,(t>>1)*0x10000+e*256+(t&1)*128+4*bank,crc[(12+t)*256+e])
for t in range(4):
    for hi in range(2):
        for nib in range(16):
            for bank in range(32):
                struct.pack_into('<I',lds,0x20000+t*4096+nib*256+hi*128+4*bank,crc[(28+t)*256+(nib<<4 if hi else nib)])
def perm(a,b,sel):
    comb=b | (a<<32); r=0
    for i in range(4):
        s=(sel>>(8*i))&0xff
        if s==0x0c: v=0
        elif s<8: v=(comb>>(8*s))&0xff
        else: raise
        r|=v<<(8*i)
    return r
def rd(a): return struct.unpack_from('<I',lds,a)[0]
def BYT(x,k,lb): return rd(perm(x,lb,0x0c000000|(0x00020000 if k>=2 else 0x000c0000)|((4+k)<<8)) + (k&1)*128)
def NIBS(t,h,xm,lb): return rd(perm(xm,lb,0x0c030000|((4+t)<<8)) + t*4096+h*128)
def step4x(x,w,lb): return BYT(x,0,lb)^BYT(x,1,lb)^BYT(x,2,lb)^BYT(x,3,lb)^w
def shift(A,lb):
    xl=A&0x0f0f0f0f; xh=(A>>4)&0x0f0f0f0f; r=0
    for t in range(4): r^=NIBS(t,0,xl,lb)^NIBS(t,1,xh,lb)
    return r
seg=os.urandom(32768)
w=np.frombuffer(seg,dtype='<u4')
raw=0
for lane in range(64):
    lb=((lane&31)<<2)|0x10000|0x2000000
    A=0
    for r in range(8):
        base=(4096*r+64*lane)//4
        words=[int(v) for v in w[base:base+16]]
        x=words[0]
        for i in range(1,16): x=step4x(x,words[i],lb)
        A=step4x(x,shift(A,lb),lb)
    raw^=mulmod(xpow8(64*(63-lane)),A)
K=mulmod(xpow8(32768),0xffffffff)
got=(~(K^raw))&0xffffffff
# reference crc32c
c=0xffffffff
for b in seg: c=T[(c^b)&0xff]^(c>>8)
print(hex(got),hex(c^0xffffffff), got==(c^0xffffffff))
