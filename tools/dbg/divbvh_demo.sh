# lanes of one wave on different BVHs (user_kernels divbvh) in every user-kernel build
for b in user_kernels uk_defer uk_share uk_oca uk_cut; do
  timeout -k 10 60 build/tests/$b divbvh 200 333 181 /tmp 3; echo "$b rc=$?"
done
exit 0
