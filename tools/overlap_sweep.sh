B=3d-wave-equation-mpi-cuda_amd/build/wave3d
for d in 2,2,2 8,1,1; do for o in "" "--no-overlap"; do
 echo -n "dims=$d ov=${o:-on} "; timeout -k 10 120 $B 1024 8 pi pi pi 1 100 --ranks 8 --dims $d $o --repeat 3 --warmup 1 --json --format none --quiet || exit 1
done; done
