export TMPDIR=/tmp
export AKR_HIP_LIB=$PWD/tools/experiments/lib/libakr_hip_wave_sort.so   # tools/experiments/build.sh wave_sort
S="python -u tools/sort_probe.py"
PMC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
tools/gpu_session.sh \
 "soup 400 $S --scene soup --spp 32 --configs path=0 path=0,wave_sort=3 path=0,wave_sort=3,wave_sort_shadow=1 path=0,wave_sort=4,wave_sort_shadow=2" \
 "soup8 300 $S --scene soup --spp 128 --split 8 --rank 0 --configs path=0 path=0,wave_sort=3 path=0,wave_sort=3,wave_sort_shadow=1" \
 "hall 400 $S --scene hall --spp 16 --configs path=0 path=0,wave_sort=3 path=0,wave_sort=4 path=0,wave_sort=3,wave_sort_shadow=1 path=0,wave_sort=3,wave_sort_shadow=2" \
 "cornell 200 $S --scene cornell --spp 64 --configs path=0 path=0,wave_sort=3 path=0,wave_sort=3,wave_sort_shadow=1" \
 "pmcsoupoff 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/pmc_soup_off -o run -- python3 tools/sort_probe.py --scene soup --spp 8 --repeat 1 --no-count --configs path=0" \
 "pmcsoupon 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/pmc_soup_on -o run -- python3 tools/sort_probe.py --scene soup --spp 8 --repeat 1 --no-count --configs path=0,wave_sort=3,wave_sort_shadow=1" \
 "pmchalloff 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/pmc_hall_off -o run -- python3 tools/sort_probe.py --scene hall --spp 8 --repeat 1 --no-count --configs path=0" \
 "pmchallon 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/pmc_hall_on -o run -- python3 tools/sort_probe.py --scene hall --spp 8 --repeat 1 --no-count --configs path=0,wave_sort=3,wave_sort_shadow=1"
