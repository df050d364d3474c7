cd "${GRAFT_REPO_ROOT}"
for sc in CBbunny dragon_proxy; do
  echo "## $sc"
  bash scripts/dev/ab_env.sh $sc "PT_INLINE_SA=0.02" "PT_INLINE_SA=0.01" "PT_INLINE_MAX=48" "PT_INLINE_MAX=64 PT_INLINE_SA=0.02" || exit $?
done
