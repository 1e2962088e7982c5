set -e
mkdir -p gpurun_out
for dev in 0 1; do
  for th in 1 8; do
    rm -f /dev/shm/ft.nc
    PNCX_PHASES=1 PNCX_IO_THREADS=$th timeout -k 10 60 tests/mpi/api_check c1first /dev/shm/ft.nc 1048576 32 $dev
  done
done
rm -f /dev/shm/ft.nc
