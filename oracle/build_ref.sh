#!/usr/bin/env bash
# TEST INFRASTRUCTURE: compile the reference Fortran 77 programs from their
# own sources under /root/reference into oracle/_ref/ (git-ignored).
#
# Recipe: ROCm flang -O2.  ROCm flang's runtime has no
# rand_/srand_, so a 2-line C forwarder maps them onto the GNU Fortran
# runtime's own _gfortran_rand/_gfortran_srand (libgfortran.so.4, present in
# this image under /opt/conda/lib).  Nothing is re-implemented: the RNG the
# reference uses is the real libgfortran one.
#
# Parameters are hard-coded in each reference program (e.g.
# Fortran/Square/bondc.f:67-92), so each variant is a sed-edited copy made in
# a scratch directory OUTSIDE the repository; only binaries land in
# oracle/_ref/.  Reference sources are never copied into the repo.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
FLANG=${FLANG:-/opt/rocm/lib/llvm/bin/flang}
GF=${GF:-/opt/conda/lib}
if [ ! -d "$REF/Fortran" ]; then
  echo "build_ref.sh: $REF not present; skipping reference build" >&2
  exit 0
fi
if [ ! -e "$GF/libgfortran.so.4" ]; then
  echo "build_ref.sh: $GF/libgfortran.so.4 missing; reference unbuildable" >&2
  exit 0
fi
mkdir -p "$OUT"
TMP=$(mktemp -d /tmp/percref.XXXXXX)
trap 'rm -rf "$TMP"' EXIT

cat > "$TMP/gfrand.c" <<'EOF'
/* forwarders: ROCm flang external rand_/srand_ -> libgfortran */
float _gfortran_rand(int *);
void _gfortran_srand(int *);
float rand_(int *i) { return _gfortran_rand(i); }
void srand_(int *i) { _gfortran_srand(i); }
EOF
gcc -O2 -c "$TMP/gfrand.c" -o "$TMP/gfrand.o"

# build NAME SRC [sed-expr ...]
build() {
  local name=$1 src=$2
  shift 2
  local f="$TMP/$name.f"
  cp "$REF/Fortran/$src" "$f"
  for e in "$@"; do sed -i "$e" "$f"; done
  "$FLANG" -O2 "$f" "$TMP/gfrand.o" -L"$GF" -lgfortran -Wl,-rpath,"$GF" \
    -o "$OUT/$name"
}

UNCOMMENT_VINT='/write(6,\*) (Vint(i), i = 1,(t-2\*m))/s/^C /  /'
TIGHT='s/1.00d-08,2500,iter,err/1.00d-14,200000,iter,err/'

# square bond + conductance (bondc), SURVEY.md §4.2
build sq_bondc_p50            Square/bondc.f
build sq_bondc_p60            Square/bondc.f 's/pb = 0.50d+00/pb = 0.60d+00/' "$UNCOMMENT_VINT"
build sq_bondc_p60_tight      Square/bondc.f 's/pb = 0.50d+00/pb = 0.60d+00/' "$TIGHT"
build sq_bondc_p60_pbc        Square/bondc.f 's/pb = 0.50d+00/pb = 0.60d+00/' 's/pbc = 0 /pbc = 1 /'
build sq_bondc_20x30_p55      Square/bondc.f 's/m = 50 /m = 20 /' 's/n = 50 /n = 30 /' 's/pb = 0.50d+00/pb = 0.55d+00/' 's/seed = 626504/seed = 777/'
build tri_bondc_p35           Triangular/bondc.f "$UNCOMMENT_VINT"
build tri_bondc_p35_tight     Triangular/bondc.f "$TIGHT"
build tri_bondc_p40_pbc       Triangular/bondc.f 's/pb = 0.35d+00/pb = 0.40d+00/' 's/pbc = 0 /pbc = 1 /'
# site labeling (config 1 = 64x64 ps .60)
build sq_site                 Square/site.f
build sq_site_64              Square/site.f 's/m = 50 /m = 64 /' 's/n = 50 /n = 64 /'
build sq_site_pbc             Square/site.f 's/pbc = 0 /pbc = 1 /'
build tri_site                Triangular/site.f
# mixed site-then-bond
build sq_sitebond             Square/sitebond.f
build sq_sitebond_p9          Square/sitebond.f 's/ps = 0.50d+00/ps = 0.90d+00/' 's/pb = 0.50d+00/pb = 0.60d+00/'
build tri_sitebond            Triangular/sitebond.f
# mixed bonds-then-sites (bondsite, Square/bondsite.f:182-354)
BS30='s/m = 10  /m = 30  /'
BN30='s/n = 10  /n = 30  /'
build sq_bondsite             Square/bondsite.f
build sq_bondsite_30          Square/bondsite.f "$BS30" "$BN30" 's/ps = 0.50d+00/ps = 0.80d+00/' 's/pb = 0.50d+00/pb = 0.70d+00/'
build sq_bondsite_30_pbc      Square/bondsite.f "$BS30" "$BN30" 's/ps = 0.50d+00/ps = 0.80d+00/' 's/pb = 0.50d+00/pb = 0.70d+00/' 's/pbc = 0 /pbc = 1 /'
build tri_bondsite            Triangular/bondsite.f
build tri_bondsite_30         Triangular/bondsite.f "$BS30" "$BN30" 's/ps = 0.50d+00/ps = 0.70d+00/' 's/pb = 0.50d+00/pb = 0.60d+00/'
# ensemble driver (trial seeds, pb sweep, per-step spanning)
build sq_bond_cond            Square/bond_cond.f
build sq_bond_cond_3t         Square/bond_cond.f 's/numtrials = 1 /numtrials = 3 /' 's/m = 10 /m = 12 /' 's/n = 10 /n = 12 /'
build tri_bond_cond           Triangular/bond_cond.f

build sq_bond_perc            Square/bond_perc.f
build sq_bond_perc_pbc        Square/bond_perc.f 's/pbc = 0 /pbc = 1 /' 's/m = 50 /m = 40 /' 's/n = 50 /n = 30 /'
build tri_bond_perc           Triangular/bond_perc.f
build sq_site_perc            Square/site_perc.f 's/numtrials = 1000 /numtrials = 40 /'
build tri_site_perc           Triangular/site_perc.f 's/numtrials = 1000 /numtrials = 40 /'
build sq_site_perc_pbc        Square/site_perc.f 's/numtrials = 1000 /numtrials = 40 /' 's/pbc = 0 /pbc = 1 /' 's/m = 50 /m = 36 /' 's/n = 50 /n = 44 /'
build sq_sb_perc              Square/sb_perc.f 's/pscount = 42 /pscount = 4 /' 's/iter = 100/iter = 5/' 's/0.59d+00+(0.01d+00\*(i-1))/0.65d+00+(0.10d+00*(i-1))/'
build tri_sb_perc             Triangular/sb_perc.f 's/pscount = 51 /pscount = 4 /' 's/iter = 100/iter = 5/' 's/0.50d+00+(0.01d+00\*(i-1))/0.60d+00+(0.10d+00*(i-1))/'
build sq_bs_perc              Square/bs_perc.f 's/pbcount = 71 /pbcount = 5 /' 's/iter = 1000/iter = 8/' 's/0.30d+00+(0.01d+00\*(i-1))/0.55d+00+(0.10d+00*(i-1))/'
build tri_bs_perc             Triangular/bs_perc.f 's/pbcount = 71 /pbcount = 5 /' 's/iter = 1000/iter = 8/' 's/0.30d+00+(0.01d+00\*(i-1))/0.55d+00+(0.10d+00*(i-1))/'
# Route 1 of INTEGRATION.md (link check, CPU side): the reference program with
# its embedded Numerical Recipes block (from SUBROUTINE sprsin to the end of
# the file: Square/bondc.f:723-917, Square/bond_cond.f:623-818) removed,
# linked against libperc's NR symbols (sprsin_, linbcg_, dsprsax_, ...) and
# its own COMMON /mat/.  Running it needs a GPU; the compiled reference never
# travels to the GPU box, so these binaries only prove the relink.
PERC_LIB=${PERC_LIB:-$HERE/../percolation_amd}
build_nr() {
  local name=$1 src=$2
  shift 2
  local f="$TMP/$name.f"
  cp "$REF/Fortran/$src" "$f"
  for e in "$@"; do sed -i "$e" "$f"; done
  sed -i '/SUBROUTINE sprsin/,$d' "$f"
  "$FLANG" -O2 "$f" "$TMP/gfrand.o" -L"$PERC_LIB" -lperc -Wl,-rpath,"$PERC_LIB" \
    -L"$GF" -lgfortran -Wl,-rpath,"$GF" -o "$OUT/$name"
}
if [ -e "$PERC_LIB/libperc.so" ]; then
  build_nr nr_sq_bondc        Square/bondc.f
  build_nr nr_sq_bondc_p60    Square/bondc.f 's/pb = 0.50d+00/pb = 0.60d+00/'
  build_nr nr_sq_bond_cond    Square/bond_cond.f
  build_nr nr_tri_bondc       Triangular/bondc.f
else
  echo "build_ref.sh: $PERC_LIB/libperc.so not built; skipping the Route-1 relink" >&2
fi
echo "reference binaries in $OUT"
