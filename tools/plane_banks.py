#!/usr/bin/env python3
"""LDS bank-conflict simulation of the GDN backward's split-plane layouts (csrc/gdn_fused.hip pl_sw): the
dx GEMM's ds_read_b128 fragments, the dgamma GEMM's ds_read_b64_tr_b16 reads and gdn_bwd_x3w_kernel's phase-A
ds_write_b64 stores, with the lane groups and bank moduli of MI355X_MICROARCH.md section LDS.  Prints the worst
n-way conflict of each access for the old and the current swizzle."""
C=192
def pl_sw_old(m): return (((m>>1)&1)<<2) | (((m>>2)&1)<<1)
def pl_sw_new(m): return (((m>>1)&1)<<2) | ((4-(m>>2))&3)
def off(m,n,sw): return m*C + (((n>>3)^sw(m))<<3) + (n&7)   # bf16 element offset
b128_groups=[[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
b128_groups+= [[x+32 for x in g] for g in b128_groups]
def conflicts(addr_dwords_per_lane, groups, nbanks):
    worst=1
    for g in groups:
        cnt={}
        for l in g:
            for d in addr_dwords_per_lane[l]:
                b=d%nbanks; cnt.setdefault(b,set()).add(d)
        worst=max(worst,max(len(v) for v in cnt.values()))
    return worst
def simulate(sw):
    """(worst n-way of the dx b128 fragment reads, of the tr reads, of the phase-A b64 stores)"""
    # (1) dx A/B fragment b128: lane (li,lg): row li, channels 32s+8lg..+7
    w1=1
    for s in range(6):
        A=[]
        for lane in range(64):
            li,lg=lane&15,lane>>4
            e=off(li,32*s+8*lg,sw); A.append([e//2+k for k in range(4)])
        w1=max(w1,conflicts(A,b128_groups,64))
    # (2) tr reads: lane: row tr_row=8*(lane>>5)+(li>>2) (+4 for hi), col c0+16*((lane>>4)&1)+4*(li&3), 2 dwords
    w2=1
    for c0 in range(0,192,32):
        for hi in (0,4):
            A=[]
            for lane in range(64):
                li=lane&15; r=8*(lane>>5)+(li>>2)+hi; c=c0+16*((lane>>4)&1)+4*(li&3)
                e=off(r,c,sw); A.append([e//2,e//2+1])
            w2=max(w2,conflicts(A,[list(range(32)),list(range(32,64))],64))
    # (3) phase A writes b64: lane (li,lg) in wave w: row li, channels 48w+4lg+16j..+3 ; groups 4x16 contiguous, banks mod 32
    w3=1
    for w in range(4):
        for j in range(3):
            A=[]
            for lane in range(64):
                li,lg=lane&15,lane>>4
                e=off(li,48*w+4*lg+16*j,sw); A.append([e//2,e//2+1])
            w3=max(w3,conflicts(A,[list(range(16*g,16*g+16)) for g in range(4)],32))
    return w1,w2,w3


if __name__ == "__main__":
    for name,sw in (('old',pl_sw_old),('new',pl_sw_new)):
        w1,w2,w3=simulate(sw)
        print(name,'b128 dx frag',w1,'tr',w2,'phaseA b64 write',w3)
